set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r01e
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01e/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r01e/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u bench.py --config 5 --sweep=0,1,2,3,5 --steps 20 --warmup 3 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u bench.py --config 2 --sweep=-1,0,3,4 --steps 30 --warmup 3 2>&1 | grep -v amdgpu.ids
