"""Writes tests/golden/bedmap_drift.json: bedmap inputs whose decimal scores make the
reference's ONE running double (AverageVisitor.hpp:46-54, reset only in End() :64-67)
differ from the exact per-row mean, with the expected output.

The expected bytes come from oracle/bedmap_oracle.c, the plain-C restatement of the
reference's sweep + fixWindow event order with the same `sum_ += x` / `sum_ -= x`
doubles (SURVEY.md §7 "hard parts": the reference prints 2|0.350001 where the exact mean
is 0.350000 on such input). The fixture is data (inputs + expected output); rerun this
script after an oracle change and review the diff.
"""
import json
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = [
    # a huge score enters and leaves next to a small one: the residual of the rounding
    # stays in sum_ and shows in the next rows' means
    {"name": "mixed_magnitude_residual",
     "ref": "chr1\t0\t10\nchr1\t20\t30\nchr1\t40\t50\n",
     "map": "chr1\t0\t10\ta\t0.1\nchr1\t1\t10\tb\t1e11\nchr1\t20\t30\tc\t0.3\n"
            "chr1\t21\t30\td\t0.4\nchr1\t40\t50\te\t0.25\n",
     "args": ["--count", "--mean"]},
    {"name": "drift_0.350001",
     "ref": "chr1\t0\t10\nchr1\t20\t30\n",
     "map": "chr1\t0\t10\tb\t5e10\nchr1\t1\t10\ta\t0.9\nchr1\t20\t30\tc\t0.3\n"
            "chr1\t21\t30\td\t0.4\n",
     "args": ["--count", "--mean"]},
    # equal rows ordered by id + remainder (CoordRestAddressCompare), not by file order
    {"name": "equal_rows_rest_order",
     "ref": "chr1\t0\t100\nchr1\t5\t8\nchr1\t50\t60\n",
     "map": "chr1\t10\t20\tz\t0.1\nchr1\t10\t20\ta\t1e17\nchr1\t10\t20\tm\t-1e17\nchr1\t55\t56\tq\t0.7\n",
     "args": ["--sum", "--mean", "--variance", "--stdev", "--cv", "--prec", "10"]},
]


def main():
    exe = os.path.join(ROOT, "oracle", "build", "bedmap_oracle")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    out = []
    with tempfile.TemporaryDirectory() as td:
        for c in CASES:
            pr, pm = os.path.join(td, "r.bed"), os.path.join(td, "m.bed")
            open(pr, "w").write(c["ref"])
            open(pm, "w").write(c["map"])
            res = subprocess.run([exe, *c["args"], pr, pm], stdout=subprocess.PIPE, check=True)
            out.append(dict(c, expect=res.stdout.decode()))
    path = os.path.join(ROOT, "tests", "golden", "bedmap_drift.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    for c in out:
        print(c["name"], repr(c["expect"]))


if __name__ == "__main__":
    main()
