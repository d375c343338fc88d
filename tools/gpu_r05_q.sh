#!/bin/bash
# Round-5 GPU call W (and Q before it): full GPU suite, smoke, and the driver's default bench line on
# the current build (lone queries at two workgroups per CU, mixed-k coalescing,
# native host-API callers).
set -o pipefail
O=gpurun_out/r05final4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 900 python -u bench.py > $O/bench.log 2> $O/bench.err || exit 3
grep '^{' $O/bench.log | tail -1 > $O/bench.json
