set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r01f
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01f/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r01f/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r01f/bench5.json
