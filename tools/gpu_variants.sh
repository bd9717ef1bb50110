# Bench d12 / d14 for each in-tree library variant named in $DSL_VARIANTS (tools/build_variant.sh;
# "default" = the product library).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do
for V in $DSL_VARIANTS; do
  LV=$V; [ "$V" = default ] && LV=
  DSL_LIB_VARIANT=$LV timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/v12_$V.json
  DSL_LIB_VARIANT=$LV timeout -k 10 300 python3 bench.py --no-cpu-baseline --depth 14 > gpurun_out/v14_$V.json
  echo "$V: $(python3 -c "import json; a=json.load(open('gpurun_out/v12_$V.json')); b=json.load(open('gpurun_out/v14_$V.json')); print(a['value'], a['roofline']['avg_launch_ms'], b['value'], b['roofline']['avg_launch_ms'])")"
done
done
