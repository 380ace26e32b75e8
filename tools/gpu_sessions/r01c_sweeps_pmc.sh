set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r01c
timeout -k 10 200 python -u bench.py --config 2 --sweep=-1,0,1,2,3,4,5 --steps 30 --warmup 5 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r01c/sweep2.jsonl &&
timeout -k 10 200 python -u bench.py --config 3 --sweep=-1,0,1,2,3,4,5 --steps 30 --warmup 5 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r01c/sweep3.jsonl &&
timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 1 --cpu-seconds 5 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r01c/bench5.json &&
tools/gpu_pmc.sh r01c 2 "EncCT<2, 1>" 1610612736
