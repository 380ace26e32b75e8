set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r01j
export CESS_DIST_BACKEND=gloo CESS_DEVICE=0
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/r01j/bench2.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/r01j/bench2.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/degraded_bench.py --nseg 16 2>&1 | grep -v amdgpu
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/degraded_bench.py --nseg 16 --frag-mib 2 > gpurun_out/r01j/deg2.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/r01j/deg2.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29513 tools/degraded_bench.py --nseg 12 --frag-mib 1 --data-shards 4 --parity-shards 2 > gpurun_out/r01j/deg3.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/r01j/deg3.log | tail -3; exit $rc
