#!/bin/bash
# Round-4 GPU session: parity suite + smoke, the default bench line (N = 1), and the one-GPU
# rehearsal of the multi-GPU line (two ranks sharing GPU 0 over gloo). Stops at the first
# crash / abort / timeout; a failing pytest (rc 1) does not stop the later steps.
# usage: tools/gpu_r4.sh <tag> [steps: any of tests,bench,gpus2]
set -u
TAG=${1:-r04}; WHAT=${2:-tests,bench,gpus2}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # step <name> <timeout> cmd...
  local name=$1 tmo=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
case ",$WHAT," in *,tests,*)
  step pytest_gpu 600 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 120 --timeout-method thread
  step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()";;
esac
case ",$WHAT," in *,bench,*)
  step bench 400 python -u bench.py;;
esac
case ",$WHAT," in *,gpus2,*)
  CESS_DIST_BACKEND=gloo CESS_DEVICE=0 step bench_gpus2_gloo 400 python -u bench.py --gpus 2 --steps 20;;
esac
echo done
