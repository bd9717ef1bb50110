# Cost probes: bench d12/d14 with the product library and with each cost-probe variant in
# $DSL_VARIANTS (one kernel component executed twice; the time difference is that component).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for V in "" $DSL_VARIANTS; do
  DSL_LIB_VARIANT=$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 > gpurun_out/x12_$V.json
  DSL_LIB_VARIANT=$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --depth 14 --steps 3 > gpurun_out/x14_$V.json
  python3 -c "
import json
a=json.load(open('gpurun_out/x12_$V.json')); b=json.load(open('gpurun_out/x14_$V.json'))
print('%-12s d12 %.3f ms (klevel %.4f)  d14 %.3f ms (klevel %.4f)' % ('$V' or 'base', a['ms_per_step'], a['roofline']['avg_launch_ms']*a['roofline']['launches'], b['ms_per_step'], b['roofline']['avg_launch_ms']*b['roofline']['launches']))"
done
