# Round-4 timeline run: per-level k_level durations (kernel trace) of C5 d12 and the timeline
# variant's per-phase real-time marks of workgroup 0 (DSL_TIMELINE build).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04_${RUN:-tl}
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt1 -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/ktb1.json 2> $OUT/kt1.err
python3 tools/level_times.py $OUT/kt1/run_kernel_trace.csv | tee -a $OUT/levels.txt
DSL_LIB_VARIANT=timeline timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/tl.json 2> $OUT/tl.err
grep -E "^\[timeline\]" $OUT/tl.err | tail -12 | cut -c1-300
