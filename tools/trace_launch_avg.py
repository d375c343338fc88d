#!/usr/bin/env python3
"""Checks a bench line's `roofline.avg_launch_us` against a rocprofv3 kernel
trace of the same run: the average duration of the LAST `launches`
dispatches of the headline kernel (the timed region; the warm-up dispatches
come first), the whole-trace average rocprofv3 --stats reports, and the frac
each gives.

Usage: python tools/trace_launch_avg.py <kernel_trace.csv> <bench.json> [--kernel scan_f32_stream_kernel]
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--kernel", default="scan_f32_stream_kernel")
    a = ap.parse_args()
    line = [ln for ln in open(a.bench) if ln.startswith("{")][-1]
    b = json.loads(line)
    rf = b["roofline"]
    n = int(rf["launches"])
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(a.trace))
            if a.kernel in r["Kernel_Name"]]
    timed = durs[-n:]
    avg_t = sum(timed) / len(timed) / 1e3
    avg_all = sum(durs) / len(durs) / 1e3
    by = rf["algorithmic_bytes_per_launch"]
    print(json.dumps({
        "kernel": a.kernel, "dispatches_in_trace": len(durs), "timed_dispatches": len(timed),
        "trace_avg_us_timed": round(avg_t, 2), "trace_avg_us_all": round(avg_all, 2),
        "bench_avg_launch_us": rf["avg_launch_us"],
        "rel_diff_timed": round(avg_t / rf["avg_launch_us"] - 1, 4),
        "frac_from_trace_timed": round(by / (avg_t * 1e-6) / 1e9 / rf["peak"], 4),
        "frac_in_bench_line": rf["frac"],
        "gpu_clock": rf.get("gpu_clock"),
    }))


if __name__ == "__main__":
    main()
