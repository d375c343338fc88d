#!/usr/bin/env python3
"""Checks a bench line's `roofline.avg_launch_us` against a rocprofv3 kernel
trace of the same run.  The headline kernel's timed dispatches are the
bench's 16-query launches over the 1M-row corpus: the same kernel symbol also
runs the no-reuse leg (4M rows, ~4x longer), the host-API single-query calls
(one query, ~15x shorter) and, with other template arguments, the configs.
So the timed window is found by shape: dispatches of the exact symbol whose
duration lies within 0.6-1.6x the bench's own average, in trace order; the
first `warmup` of them are the warm-up, the next `launches` the timed region.

Usage: python tools/trace_launch_avg.py <kernel_trace.csv> <bench.json>
           [--kernel 'scan_f32_stream_kernel<0, 128, 1>'] [--warmup 5] [--keep out.csv]
--keep writes the matching dispatches (a few hundred rows) so the evidence
survives deleting the full trace.
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--kernel", default="scan_f32_stream_kernel<0, 128, 1>")
    ap.add_argument("--warmup", type=int, default=-1, help="warm-up launches (default: the line's `warmup`)")
    ap.add_argument("--keep", default="")
    a = ap.parse_args()
    line = [ln for ln in open(a.bench) if ln.startswith("{")][-1]
    b = json.loads(line)
    rf = b["roofline"]
    n = int(rf["launches"])
    warm = a.warmup if a.warmup >= 0 else int(b.get("warmup", 0))
    avg_b = float(rf["avg_launch_us"]) * 1e3  # ns
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    shaped = [r for r in rows if 0.6 * avg_b <= int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) <= 1.6 * avg_b]
    timed = shaped[warm:warm + n]
    if a.keep:
        with open(a.keep, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(shaped)
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed]
    avg_t = sum(durs) / max(1, len(durs)) / 1e3
    by = rf["algorithmic_bytes_per_launch"]
    print(json.dumps({
        "kernel": a.kernel, "dispatches_of_symbol": len(rows), "dispatches_of_headline_shape": len(shaped),
        "warmup_skipped": warm, "timed_dispatches": len(timed),
        "trace_avg_us_timed": round(avg_t, 2), "trace_min_us": round(min(durs) / 1e3, 2) if durs else None,
        "trace_max_us": round(max(durs) / 1e3, 2) if durs else None,
        "bench_avg_launch_us": rf["avg_launch_us"],
        "rel_diff_timed": round(avg_t / rf["avg_launch_us"] - 1, 4) if durs else None,
        "frac_from_trace_timed": round(by / (avg_t * 1e-6) / 1e9 / rf["peak"], 4) if durs else None,
        "frac_in_bench_line": rf["frac"],
        "gpu_clock": rf.get("gpu_clock"),
    }))


if __name__ == "__main__":
    main()
