#!/bin/bash
# Run the steps of a step file on the GPU box, one line each: `<name> <timeout-s> <command...>`
# (blank lines and # comments skipped). Output of step <name> goes to gpurun_out/<tag>/<name>.log.
# Stops at the first crash, abort or timeout (exit codes other than 0/1).
# usage: tools/gpu_steps.sh <tag> <step-file>
set -u
TAG=$1; FILE=$2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp OUT
while read -r name tmo cmd; do
  [ -z "${name:-}" ] && continue
  case "$name" in \#*) continue ;; esac
  echo "== $name: $cmd"
  timeout -k 10 "$tmo" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done < "$FILE"
echo done
