#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950: TCC has 4 slots, they cost 3 + 2).

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE is in KiB and reports half the bytes of
a wide coalesced streaming read on gfx950, so read bytes = 2 * FETCH_SIZE * 1024;
WRITE_SIZE is exact for 16-byte streaming stores: write bytes = WRITE_SIZE * 1024.

usage: python tools/pmc_traffic.py <fetch pass dir> <write pass dir> <out.json>
The JSON maps kernel -> {"bytes": read+write per launch, "read": ..., "write": ...,
"launches": n}; bench.py reports "traffic" for its dominant kernel from it.
"""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = collections.defaultdict(dict)  # kernel -> dispatch -> value
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") != counter:
                    continue
                k = r["Kernel_Name"].split("(")[0].strip()
                if k.startswith("void "):
                    k = k[5:]
                disp = (fn, r.get("Dispatch_Id"))
                vals[k][disp] = vals[k].get(disp, 0.0) + float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in vals.items()}


def main(fetch_dir, write_dir, out):
    fe = per_kernel(fetch_dir, "FETCH_SIZE")
    wr = per_kernel(write_dir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fe) | set(wr)):
        rd = 2.0 * fe.get(k, (0.0, 0))[0] * 1024
        wb = wr.get(k, (0.0, 0))[0] * 1024
        res[k] = {"bytes": round(rd + wb), "read": round(rd), "write": round(wb),
                  "launches": max(fe.get(k, (0, 0))[1], wr.get(k, (0, 0))[1])}
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["bytes"])[:12]:
        print(f"{k:<28} {v['bytes'] / 1e6:10.1f} MB/launch (r {v['read'] / 1e6:.1f} w {v['write'] / 1e6:.1f})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
