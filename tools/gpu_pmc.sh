# Round-2 profile of bench.py's workload: kernel trace + stats, then one rocprofv3 --pmc pass per
# counter group (HBM bytes, atomics at L2 / memory, L2 hit rate, DRAM vs Infinity-Cache reads, SQ).
# usage: bash tools/gpu_pmc.sh TAG [bench args...]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d $OUT/kt -o run -- python3 bench.py --no-cpu-baseline "$@" > $OUT/kt_bench.json 2> $OUT/kt.err
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_ATOMIC_sum TCC_EA0_WRREQ_ATOMIC_DRAM_sum" \
         "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum" "TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_FLAT SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"; do
  N=$(echo $P | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex 'k_level' -f csv -T -d $OUT/pmc_$N -o run -- python3 bench.py --no-cpu-baseline "$@" --steps 1 --warmup 0 > $OUT/pmc_$N.json 2> $OUT/pmc_$N.err
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.json
echo done $TAG
