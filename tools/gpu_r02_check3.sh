# GPU suite + per-level comparison of the product library against a saved previous build.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
DSL_VARIANTS="default scan1" bash tools/gpu_r02_vlevels.sh scan1
DSL_VARIANTS="default scan1" bash tools/gpu_r02_vlevels.sh scan1_14 --depth 14
echo done
