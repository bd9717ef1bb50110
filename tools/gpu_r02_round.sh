# Round-2 evidence run: PMC/kernel-stat profiles at d12 and d14, then a 2-rank RCCL rehearsal on one device.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_r02_prof.sh d12
bash tools/gpu_r02_prof.sh d14 --depth 14
export TMPDIR=/tmp
DSL_BENCH_SHARE_DEVICE=1 timeout -k 10 180 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rccl2.json 2> gpurun_out/rccl2.err
echo rccl-ok
