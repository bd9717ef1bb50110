# GPU step: selected test files (a failing assert does not stop the profile steps; a timeout,
# abort or fault does), then the round-2 profiles of C5 d12 / d14 and a full bench line.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/t_step.log 2>&1
rc=$?
tail -n 3 gpurun_out/t_step.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ -n "$NOPROF" ] && exit $rc
bash tools/gpu_r02_prof.sh d12 --depth 12 && bash tools/gpu_r02_prof.sh d14 --depth 14 && timeout -k 10 300 python3 bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
