set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r01i
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r01i/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r01i/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --config 6 --sweep=-1 --steps 10 --warmup 2 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u bench.py --config 3 --generic --sweep=-1 --steps 10 --warmup 2 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u bench.py --config 2 --generic --sweep=-1 --steps 10 --warmup 2 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u bench.py --config 5 --generic --sweep=-1 --steps 10 --warmup 2 2>&1 | grep -v amdgpu.ids
