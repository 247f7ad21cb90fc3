"""Starch inputs through the drop-in front-ends on the GPU: every command gives the same
bytes on an archive as on the BED it holds (the reference's own archives, tests/golden/starch/;
the reference reads Starch wherever it reads BED files, AllocateIterator_BED_starch.hpp:62)."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

D = os.path.join(os.path.dirname(__file__), "golden", "starch")
MANIFEST = [m for m in json.load(open(os.path.join(D, "manifest.json")))
            if m["bed"] != "statistics__reference_bedmap_motifs.bed"]  # hand-edited BED (test_starch.py)


def run(binary, args):
    r = subprocess.run([binary] + args, capture_output=True)
    return r.returncode, r.stdout, r.stderr


@pytest.mark.parametrize("m", MANIFEST, ids=lambda m: m["starch"])
def test_bedops_on_archive_equals_bed(gpu_bin, m):
    st, bed = os.path.join(D, m["starch"]), os.path.join(D, m["bed"])
    for args in (["--everything"], ["--ec", "--merge"]):
        a = run(gpu_bin["bedops"], args + [st])
        b = run(gpu_bin["bedops"], args + [bed])
        assert a == b, (args, a[2][:200])
    a = run(gpu_bin["bedops"], ["--intersect", st, bed])
    b = run(gpu_bin["bedops"], ["--intersect", bed, bed])
    assert a == b


def test_bedmap_and_closest_on_archives(gpu_bin, tmp_path):
    ref = os.path.join(D, "statistics__reference_bedmap_reference")
    mp = os.path.join(D, "statistics__reference_bedmap_map")
    for ops in (["--echo", "--count", "--mean", "--max-element"], ["--echo-map-id", "--bases-uniq"]):
        a = run(gpu_bin["bedmap"], ops + ["--skip-unmapped", ref + ".starch", mp + ".starch"])
        b = run(gpu_bin["bedmap"], ops + ["--skip-unmapped", ref + ".bed", mp + ".bed"])
        assert a == b and a[0] == 0, (ops, a[2][:200])
    from bedops_amd.engine import starch_to_bed
    pa = os.path.join(D, "set-operations__reference_bedextract_target.starch")
    bed = tmp_path / "t.bed"
    bed.write_bytes(starch_to_bed(open(pa, "rb").read()))
    for pair in ((pa, pa), (str(bed), pa)):
        a = run(gpu_bin["closest"], ["--closest", "--dist", pair[0], pair[1]])
        b = run(gpu_bin["closest"], ["--closest", "--dist", str(bed), str(bed)])
        assert a == b and a[0] == 0
