# FETCH_SIZE / WRITE_SIZE calibration passes over tools/hbm_calib (built beforehand, in-tree).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
timeout -k 10 120 tools/_build/hbm_calib > gpurun_out/calib/plain.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/calib/fetch -o run -- tools/_build/hbm_calib > gpurun_out/calib/fetch.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/calib/write -o run -- tools/_build/hbm_calib > gpurun_out/calib/write.txt 2>&1
python3 tools/hbm_calib.py gpurun_out/calib
