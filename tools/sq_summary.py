#!/usr/bin/env python3
"""Per-kernel SQ counters from rocprofv3 --pmc passes (tools/gpu_r04_pmc_sq.sh): each
counter summed over a kernel's dispatches, divided by its dispatches, and per wave.
usage: python tools/sq_summary.py <pass dir> [<pass dir> ...] [--kernel SUBSTR]"""
import collections
import csv
import glob
import os
import sys


def main(argv):
    ksub = None
    if "--kernel" in argv:
        i = argv.index("--kernel")
        ksub = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    val = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in argv:
        for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(fn) as f:
                for r in csv.DictReader(f):
                    k = r["Kernel_Name"].split("(")[0].strip()
                    if ksub and ksub not in k:
                        continue
                    val[k][r["Counter_Name"]] += float(r["Counter_Value"])
                    disp[k].add((fn, r.get("Dispatch_Id")))
    for k, c in sorted(val.items(), key=lambda kv: -kv[1].get("SQ_WAVES", 0)):
        n = max(1, len(disp[k]) // max(1, sum(1 for _ in c)))
        waves = c.get("SQ_WAVES", 0)
        print(f"== {k}  (waves {waves:.0f})")
        for name, v in sorted(c.items()):
            print(f"   {name:<24} {v:14.0f}   per wave {v / waves if waves else 0:10.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
