# Round-4 IR gap: per-phase and per-class handler cycles (libdslabs_hip_phases) of C5 d12 on the
# hand-written and IR-generated Multi-Paxos, and workgroup 0's per-level timeline (libdslabs_hip_timeline)
# of the IR form; then the IR GPU tests (C5 d12 sharded, lab3 argument predicates).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04_irph
mkdir -p $OUT
for W in multipaxos multipaxos_ir; do
  DSL_LIB_VARIANT=phases timeout -k 10 120 python3 bench.py --workload $W --no-cpu-baseline --steps 1 --warmup 0 > $OUT/ph_$W.json 2> $OUT/ph_$W.err
  grep -E "^\[(phases|phcls)\]" $OUT/ph_$W.err | tail -24 > $OUT/ph_$W.txt
  DSL_LIB_VARIANT=timeline timeout -k 10 120 python3 bench.py --workload $W --no-cpu-baseline --steps 2 --warmup 1 > $OUT/tl_$W.json 2> $OUT/tl_$W.err
  grep -E "^\[timeline\]" $OUT/tl_$W.err | tail -12 | cut -c1-400 > $OUT/tl_$W.txt
done
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_ir.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
