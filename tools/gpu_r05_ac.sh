#!/bin/bash
# Round-5 GPU call AC: CPU cost of a kernel launch call by argument size.
set -o pipefail
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 120 ./tools/launch_probe > $O/launch_probe.jsonl 2> $O/launch_probe.err || exit 1
