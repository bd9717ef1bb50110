# Round-4 IR / Sender run: C5 d12 per-level k_level durations of the hand-written and IR-generated
# Multi-Paxos on the product library (base) and on the variants in $VARS (default: the shift-register
# Sender, libdslabs_hip_shift),
# then per-class handler cycles and per-phase cycles (libdslabs_hip_phases) for both protocols.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04_ir}
mkdir -p $OUT
for r in 1 2; do
for V in ${VARS:-base shift}; do
for W in multipaxos multipaxos_ir; do
  LV=$V; [ "$V" = base ] && LV=
  DSL_LIB_VARIANT=$LV timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $OUT/kt_${V}_${W}_$r -o run -- python3 bench.py --workload $W --no-cpu-baseline --steps 3 --warmup 1 > $OUT/b_${V}_${W}_$r.json 2> $OUT/e_${V}_${W}_$r.err
  echo "$V $W/$r: $(python3 tools/level_times.py $OUT/kt_${V}_${W}_$r/run_kernel_trace.csv)" | tee -a $OUT/levels.txt
done
done
done
[ -n "$NOPH" ] && exit 0
for W in multipaxos multipaxos_ir; do
  DSL_LIB_VARIANT=phases timeout -k 10 120 python3 bench.py --workload $W --no-cpu-baseline --steps 1 --warmup 0 > $OUT/ph_$W.json 2> $OUT/ph_$W.err
  grep -E "^\[(phases|phcls)\]" $OUT/ph_$W.err | tail -24 > $OUT/ph_$W.txt
done
