# Timeline variant (WG 0 marks only) on C5 d12, then the synthetic waves-per-SIMD variants.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04_tl2
mkdir -p $OUT
DSL_LIB_VARIANT=timeline timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/tl.json 2> $OUT/tl.err
grep -E "^\[timeline\]" $OUT/tl.err | tail -12 | cut -c1-400
TAG=synwaves2 VN=2 VARIANTS="w5 w6" BENCH_ARGS="--workload synthetic --steps 5 --warmup 1" bash tools/gpu_variants_bench.sh
