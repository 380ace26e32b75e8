#!/bin/bash
# Rehearse the multi-GPU bench paths (default line's degraded-gather leg, config 4) with several
# ranks on one GPU over gloo (RCCL needs one GPU per rank; the driver's scaling run uses it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/multirank
export CESS_DIST_BACKEND=gloo CESS_DEVICE=0
for n in 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 2 \
    > gpurun_out/multirank/c2_n$n.json 2> gpurun_out/multirank/c2_n$n.err || { tail -20 gpurun_out/multirank/c2_n$n.err; exit 1; }
  tail -c 700 gpurun_out/multirank/c2_n$n.json; echo
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29510 bench.py --gpus 2 --config 4 --steps 2 --warmup 1 \
  > gpurun_out/multirank/c4_n2.json 2> gpurun_out/multirank/c4_n2.err || { tail -20 gpurun_out/multirank/c4_n2.err; exit 1; }
tail -c 900 gpurun_out/multirank/c4_n2.json
