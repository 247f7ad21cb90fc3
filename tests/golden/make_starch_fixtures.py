"""Copies the reference's own Starch archives that come with the BED they hold into
tests/golden/starch/ (data only) and writes manifest.json pairing them. Sources: the
conversion tests (applications/bed/conversion/src/tests/*: each tool's expected BED and its
Starch output, bzip2 and gzip) and the documentation assets
(docs/assets/reference/*/reference_*.{bed,starch}). Run from the repo root with the
reference at /root/reference; the copies are committed, so tests never read the reference."""
import glob
import json
import os
import shutil

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(__file__), "starch")


def pairs():
    t = os.path.join(REF, "applications/bed/conversion/src/tests")
    for st in sorted(glob.glob(os.path.join(t, "*", "*.starch"))):
        d, b = os.path.split(st)
        stem = b[: -len(".starch")]
        for suffix in (".gzip", ".bzip2"):
            if stem.endswith(suffix):
                stem = stem[: -len(suffix)]
        bed = os.path.join(d, stem + ".bed")
        if os.path.exists(bed):
            yield st, bed
    for st in sorted(glob.glob(os.path.join(REF, "docs/assets/reference/*/*.starch"))):
        bed = st[: -len(".starch")] + ".bed"
        if os.path.exists(bed):
            yield st, bed


def main():
    os.makedirs(OUT, exist_ok=True)
    man = []
    for st, bed in pairs():
        tag = os.path.basename(os.path.dirname(st))
        a = f"{tag}__{os.path.basename(st)}"
        b = f"{tag}__{os.path.basename(bed)}"
        shutil.copyfile(st, os.path.join(OUT, a))
        shutil.copyfile(bed, os.path.join(OUT, b))
        man.append({"starch": a, "bed": b, "source": os.path.relpath(st, REF)})
    json.dump(man, open(os.path.join(OUT, "manifest.json"), "w"), indent=1)
    print(len(man), "pairs")


if __name__ == "__main__":
    main()
