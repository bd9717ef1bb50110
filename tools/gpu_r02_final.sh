# Round-2 closing run: GPU suite, smoke, bench lines and the PMC profiles of the final engine.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_r02_check2.sh
bash tools/gpu_r02_prof.sh d12
bash tools/gpu_r02_prof.sh d14 --depth 14
echo final-done
