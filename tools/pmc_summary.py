#!/usr/bin/env python3
"""Per-kernel averages of every PMC counter and the dispatch time in one or
more rocprofv3 sqlite outputs (tooling).  Usage: pmc_summary.py <dir-or-db>... [--match SUBSTR]"""
import argparse
import collections
import glob
import os
import sqlite3


def rows(db):
    con = sqlite3.connect(db)
    names = dict(con.execute("select id, name from rocpd_info_pmc"))
    ks = dict(con.execute("select id, kernel_name from rocpd_info_kernel_symbol"))
    disp = {r[0]: (ks.get(r[1], "?"), r[3] - r[2]) for r in
            con.execute("select event_id, kernel_id, start, end from rocpd_kernel_dispatch")}
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for ev, pid, v in con.execute("select event_id, pmc_id, value from rocpd_pmc_event"):
        vals[ev][names[pid]] += v
    for ev, (name, dur) in disp.items():
        yield name, dur, dict(vals.get(ev, {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    for p in a.paths:
        dbs = [p] if p.endswith(".db") else glob.glob(os.path.join(p, "**", "*.db"), recursive=True)
        for db in sorted(dbs):
            agg = collections.defaultdict(list)
            for name, dur, cv in rows(db):
                if a.match in name:
                    agg[name].append((dur, cv))
            for name, lst in sorted(agg.items(), key=lambda x: -sum(d for d, _ in x[1])):
                keys = sorted({k for _, cv in lst for k in cv})
                avg = {k: sum(cv.get(k, 0.0) for _, cv in lst) / len(lst) for k in keys}
                print(f"{os.path.basename(db)} {name[:90]} n={len(lst)} avg_us={sum(d for d, _ in lst) / len(lst) / 1e3:.1f} "
                      + " ".join(f"{k}={v:.5g}" for k, v in avg.items()))


if __name__ == "__main__":
    main()
