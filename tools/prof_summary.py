#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats output (SQLite .db or *_kernel_stats.csv)
into profiles/<name>.csv: kernel, calls, total_us, avg_us, percent.

usage: python tools/prof_summary.py <rocprof output dir or .db> <profiles/out.csv>
"""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    db = sqlite3.connect(path)
    rows = db.execute("select name, total_calls, total_duration, average, percentage "
                      "from top_kernels").fetchall()
    return [(n.split("(")[0], int(c), t, a, p) for n, c, t, a, p in rows]  # top_kernels view: microseconds


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"].split("(")[0], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                        float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return out


def main(src, dst):
    if os.path.isdir(src):
        dbs = glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
        csvs = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True)
        rows = from_csv(csvs[0]) if csvs else from_db(dbs[0])
    elif src.endswith(".db"):
        rows = from_db(src)
    else:
        rows = from_csv(src)
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for r in rows:
            w.writerow([r[0], r[1], f"{r[2]:.3f}", f"{r[3]:.3f}", f"{r[4]:.2f}"])
    for r in rows[:12]:
        print(f"{r[0]:<32} {r[1]:>6} {r[3]:>12.3f} us avg {r[4]:6.2f}%")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
