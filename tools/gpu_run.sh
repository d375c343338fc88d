#!/usr/bin/env bash
# Runs GPU steps on the gpurun box, each under its own time limit.  Stops at
# the first step that ends in a fault-class status (abort 134, segfault 139,
# timeout 124/137) -- nothing more touches the GPU after that; an ordinary
# failure (e.g. a failing assertion, status 1) does not stop later steps.
# Usage: tools/gpu_run.sh "<limit_s>:<name>:<command>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
overall=0
for spec in "$@"; do
  limit="${spec%%:*}"; rest="${spec#*:}"; name="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${limit}s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc after $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then overall=$rc; fi
  case $rc in
    124|134|137|139) echo "fault-class status $rc: stopping"; exit $rc ;;
  esac
done
exit $overall
