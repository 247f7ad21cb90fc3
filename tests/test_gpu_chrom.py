"""--chrom on regular files reads only that chromosome's lines, as the reference's
find_bed_range seek does (AllocateIterator_BED_starch.hpp:113-160): rows of other
chromosomes are never parsed, so a bad line elsewhere does not stop the command."""
import os
import random
import subprocess

import pytest

import randbed

pytestmark = pytest.mark.gpu


def test_chrom_reads_only_its_range(gpu_bin, tmp_path):
    rng = random.Random(12)
    chroms = ["chr1", "chr10", "chr2", "chrX"]
    a = randbed.rows(rng, 3000, chroms=chroms, span=5000, maxlen=60)
    b = randbed.rows(rng, 3000, chroms=chroms, span=5000, maxlen=60)
    ta, tb = randbed.text(a), randbed.text(b, rest="bed5", rng=rng)
    # a malformed line inside chr10 and an out-of-order row in chrX of file a
    la = ta.splitlines(keepends=True)
    i10 = next(k for k, ln in enumerate(la) if ln.startswith("chr10\t"))
    ix = next(k for k, ln in enumerate(la) if ln.startswith("chrX\t"))
    bad = la[:i10 + 1] + ["chr10\tnot_a_number\t5\n"] + la[i10 + 1:ix + 2] + ["chrX\t0\t1\n"] + la[ix + 2:]
    pa, pb = tmp_path / "a.bed", tmp_path / "b.bed"
    pa.write_text("".join(bad))
    pb.write_text(tb)
    for c in ("chr1", "chr2", "chr9"):
        only = tmp_path / f"a_{c}.bed"
        only.write_text("".join(ln for ln in bad if ln.split("\t")[0] == c))
        onlyb = tmp_path / f"b_{c}.bed"
        onlyb.write_text("".join(ln for ln in tb.splitlines(keepends=True) if ln.split("\t")[0] == c))
        for args in (["--merge"], ["--intersect"], ["--element-of", "1"]):
            g = subprocess.run([gpu_bin["bedops"], "--chrom", c] + args + [str(pa), str(pb)], capture_output=True)
            w = subprocess.run([gpu_bin["bedops"]] + args + [str(only), str(onlyb)], capture_output=True)
            assert g.returncode == 0, g.stderr
            assert g.stdout == w.stdout, (c, args)
        g = subprocess.run([gpu_bin["bedmap"], "--chrom", c, "--echo", "--count", "--mean", str(pa), str(pb)],
                           capture_output=True)
        w = subprocess.run([gpu_bin["bedmap"], "--echo", "--count", "--mean", str(only), str(onlyb)],
                           capture_output=True)
        assert g.returncode == 0 and g.stdout == w.stdout, (c, g.stderr)
    # the bad chromosomes themselves still fail
    g = subprocess.run([gpu_bin["bedops"], "--chrom", "chr10", "--merge", str(pa)], capture_output=True)
    assert g.returncode != 0
