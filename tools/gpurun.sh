#!/bin/bash
# Rebuild every in-tree artefact on the CPU, then hand the command to gpurun.
# usage: tools/gpurun.sh <timeout-seconds> '<command>'
set -e
cd "$(dirname "$0")/.."
python -c "import __graft_entry__ as g; g.build()" > /tmp/build.log 2>&1 || { tail -20 /tmp/build.log; exit 1; }
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
