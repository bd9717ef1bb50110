# Round-4 IR gap: instruction-issue and instruction-cache counters of k_level on C5 d12, hand-written
# vs IR-generated Multi-Paxos (one PMC pass per counter set, one search each).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04_icache
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
grep -oE "SQC_[A-Z_0-9]+|SQ_IFETCH[A-Z_]*|SQ_INSTS_[A-Z_]+|SQ_WAIT_[A-Z_]+" $OUT/counters.txt | sort -u > $OUT/names.txt || true
for W in multipaxos multipaxos_ir; do
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_WAIT_ANY SQ_IFETCH SQ_INSTS_BRANCH SQ_BUSY_CYCLES" "SQC_ICACHE_HITS SQC_ICACHE_MISSES"; do
  N=$(echo $P | tr ' ' '_' | cut -c1-30)
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex 'k_level' -f csv -d $OUT/${W}_$N -o run -- python3 bench.py --workload $W --no-cpu-baseline --steps 1 --warmup 0 > $OUT/${W}_$N.json 2> $OUT/${W}_$N.err || echo "pass $N failed for $W"
done
done
echo done
