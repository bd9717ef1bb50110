# GPU suite + smoke + default bench + kernel stats + per-level times on the product library.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 python -u bench.py --depth 14 --steps 3 --no-cpu-baseline > gpurun_out/bench14.json 2> gpurun_out/bench14.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
DSL_VARIANTS=default bash tools/gpu_r02_vlevels.sh final
echo done
