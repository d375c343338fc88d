#!/bin/bash
# One GPU call: run the named pytest files (or the whole -m gpu suite) with a
# per-test timeout, logging to gpurun_out/<tag>.log.  Usage:
#   tools/gpu_run_tests.sh TAG [pytest args...]
set -o pipefail
tag=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" \
    > "gpurun_out/$tag.log" 2>&1
rc=$?
tail -5 "gpurun_out/$tag.log"
exit $rc
