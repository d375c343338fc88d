"""The multi-GPU bench code on a one-GPU box (the driver's SCALE runs exactly
this code at N = 2, 4, 8 on an 8-GPU node): bench.py --gpus 2 --share-gpu
re-launches itself as two ranks on cuda:0 that exchange their packed top-k
blocks over gloo, and --workload slab1b deals 8 slabs to the ranks.  Each run
checks its merged results against the oracle's top-k over every shard's rows
(bench.py merge_check) -- here at sizes the host oracle finishes in seconds."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, timeout=240):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--configs", "",
                        *args], capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.parametrize("gpus", [2, 3])
def test_flat_share_gpu_exchange_and_merge(gpus):
    out = run_bench("--gpus", str(gpus), "--share-gpu", "--rows", "300000", "--steps", "3", "--warmup", "1",
                    "--s1b-rows", "4000000", "--pq-rows", "400000")
    assert out["n_gpus"] == gpus and out["value"] > 0
    assert out["merge_check"]["ok"] is True, out["merge_check"]
    # the strong-scaling legs the driver's SCALE line carries (configs[4] and configs[3]), at test sizes
    legs = out["configs"]
    if gpus == 3:
        assert "skipped" in legs["config5_1b_x_128"]
    else:
        assert legs["config5_1b_x_128"]["slabs_per_gpu"] == 8 // gpus
        assert legs["config5_1b_x_128"]["merge_check"]["ok"] is True, legs["config5_1b_x_128"]
    assert legs["config4_pq_sharded"]["merge_check"]["ok"] is True, legs["config4_pq_sharded"]
    assert legs["config4_pq_sharded"]["rows_per_gpu"] >= 400000 // gpus
    # the one-process multi-GPU leg needs N devices in one process: skipped on a shared GPU
    assert "skipped" in legs["multi_gpu_one_process"]


@pytest.mark.parametrize("gpus", [1, 2])
def test_slab1b_deal_merge(gpus):
    args = ["--workload", "slab1b", "--rows", "4000000", "--steps", "2", "--warmup", "1", "--gpus", str(gpus)]
    if gpus > 1:
        args.append("--share-gpu")
    out = run_bench(*args)
    assert out["config"]["slabs"] == 8 and out["config"]["slabs_per_gpu"] == 8 // gpus
    assert out["merge_check"]["ok"] is True, out["merge_check"]
