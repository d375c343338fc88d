"""Where do the bf16 screen's results differ from the exact path's?  For a
few batch sizes, prints the mismatching queries, the rank where they first
differ, both sides' (id, distance) there, and the oracle's answer.
Usage: python tools/screen_debug.py [--metric cosine|dot] [--d 768]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--metric", default="cosine")
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--n", type=int, default=30_077)
    ap.add_argument("--cases", default="32:10,300:10,40:1,129:16,64:7,40:1,300:10")
    ap.add_argument("--repeat", type=int, default=3)
    args = ap.parse_args()
    import torch

    torch.cuda.init()
    from oracle import wv_oracle as orc
    from weaviate_amd._lib import KIND_F32, METRIC_COSINE, METRIC_DOT
    from weaviate_amd.device import Context, Corpus

    orc.lib()
    metric = METRIC_COSINE if args.metric == "cosine" else METRIC_DOT
    d, n = args.d, args.n
    rows = orc.synth_rows(1000 + d, 0, n, d, 0)
    qs = orc.synth_rows(1001 + d, 0, 300, d, 0)
    ctx = Context(0)
    ex = Context(0, batch_screen=0)
    a = Corpus(ctx, KIND_F32, metric, d, n)
    b = Corpus(ex, KIND_F32, metric, d, n)
    ids = np.arange(n, dtype=np.uint64)
    a.upsert(ids, rows)
    b.upsert(ids, rows)
    dead = np.array([0, 5, 64, 255, 256, 20_000, n - 1], np.uint64)
    a.delete(dead)
    b.delete(dead)
    srows = orc.normalize_rows(rows) if metric == METRIC_COSINE else rows
    for case in args.cases.split(","):
        nq, k = (int(x) for x in case.split(":"))
        bi, bd, bc = b.search(qs[:nq], k)
        for rep in range(args.repeat):
            ai, ad, ac = a.search(qs[:nq], k)
            bad = [q for q in range(nq) if not (np.array_equal(ai[q], bi[q]) and
                                                 np.array_equal(ad[q].view(np.uint32), bd[q].view(np.uint32)) and
                                                 ac[q] == bc[q])]
            rec = {"nq": nq, "k": k, "rep": rep, "mismatching_queries": len(bad), "first": bad[:12]}
            det = []
            for q in bad[:3]:
                r = int(np.argmax((ai[q] != bi[q]) | (ad[q].view(np.uint32) != bd[q].view(np.uint32))))
                qq = orc.normalize(qs[q]) if metric == METRIC_COSINE else qs[q]
                od = orc.dist_all(2 if metric == METRIC_COSINE else 1, qq, srows)
                od[dead.astype(np.int64)] = np.inf
                order = np.lexsort((np.arange(n), od))[:k]
                det.append({"q": q, "rank": r, "screen": [int(ai[q][r]), float(ad[q][r])],
                            "exact": [int(bi[q][r]), float(bd[q][r])],
                            "oracle": [int(order[r]), float(od[order[r]])],
                            "screen_ids": [int(x) for x in ai[q]], "exact_ids": [int(x) for x in bi[q]]})
            rec["detail"] = det
            print(json.dumps(rec), flush=True)
    a.destroy()
    b.destroy()
    ex.close()
    ctx.close()


if __name__ == "__main__":
    main()
