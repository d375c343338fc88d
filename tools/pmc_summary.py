#!/usr/bin/env python3
"""Per-kernel averages of every PMC counter and the dispatch time in one or
more rocprofv3 outputs, sqlite or csv (tooling).  Usage: pmc_summary.py <dir-or-db>... [--match SUBSTR]"""
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


def csv_rows(path):
    """rocprofv3 --output-format csv: one row per (dispatch, counter)."""
    import csv
    disp = {}
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    with open(path) as f:
        for r in csv.DictReader(f):
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            try:
                dur = int(r.get("End_Timestamp") or 0) - int(r.get("Start_Timestamp") or 0)
            except ValueError:
                dur = 0
            disp[d] = (r.get("Kernel_Name", "?"), dur)
            vals[d][r["Counter_Name"]] += float(r["Counter_Value"])
    for d, (name, dur) in disp.items():
        yield name, dur, dict(vals[d])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    for p in a.paths:
        dbs = [p] if p.endswith((".db", ".csv")) else (
            glob.glob(os.path.join(p, "**", "*.db"), recursive=True) +
            glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True))
        for db in sorted(dbs):
            agg = collections.defaultdict(list)
            for name, dur, cv in (csv_rows(db) if db.endswith(".csv") else rows(db)):
                if a.match in name:
                    agg[name].append((dur, cv))
            for name, lst in sorted(agg.items(), key=lambda x: -sum(d for d, _ in x[1])):
                keys = sorted({k for _, cv in lst for k in cv})
                avg = {k: sum(cv.get(k, 0.0) for _, cv in lst) / len(lst) for k in keys}
                print(f"{os.path.basename(db)} {name[:90]} n={len(lst)} avg_us={sum(d for d, _ in lst) / len(lst) / 1e3:.1f} "
                      + " ".join(f"{k}={v:.5g}" for k, v in avg.items()))


if __name__ == "__main__":
    main()
