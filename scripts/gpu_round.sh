#!/usr/bin/env bash
# Guarded GPU session: each step has its own time limit; on a fault/abort/segfault/timeout
# (exit 124/134/137/139 or >128) nothing else touches the GPU.  Test failures (exit 1) do not
# stop the later measurement steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
export TMPDIR=/tmp
step() {  # step <name> <timeout-seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== [$name] $(date +%T) $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc" | tee -a gpurun_out/steps.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "!!! fatal rc=$rc in $name: stopping GPU work" | tee -a gpurun_out/steps.log
    exit $rc
  fi
  return 0
}
