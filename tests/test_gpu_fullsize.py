"""BASELINE.json configs at full size against the genuine reference's output.

tests/golden/ref_fullsize.json holds, per bench.py workload, the rows / bytes / sha256 prefix
of the reference's own output (BEDOPS v2.4.26 built by oracle/build_ref.sh, one process on the
whole generated files; tools/pin_fullsize.py, run in the build container). Here the same
inputs are generated on the GPU box (tools/bedgen.c), put in HBM, run
through the C ABI exactly as bench.py times them, and the output text is hashed:
  bedmap         --count --mean 50M x 500M BED5          configs[2], one MI355X
  element-of     --element-of 1 200M x 200M              configs[3] (the 8-GPU config's data on one GPU)
  closest        --closest 10M x 1B                      configs[4] (the 8-GPU config's data on one GPU)
  bedmap-decimal --count --mean 5M x 50M, decimal scores (running doubles replayed)
(configs[1], 100M x 100M --intersect, is checked by bench.py after every timed run and by
tests/test_gpu_parity.py::test_intersect_and_element_of_100M_reference_hash.)
"""
import hashlib
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

with open(os.path.join(ROOT, "tests", "golden", "ref_fullsize.json")) as f:
    REF = json.load(f)


@pytest.fixture(scope="module")
def eng():
    from bedops_amd import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("name", ["element-of", "bedmap", "closest", "bedmap-decimal"])
def test_fullsize_output_matches_reference(eng, name):
    # the generated text goes in from host memory (bg_load's staging ring): torch is not
    # initialised in this process, whose HIP runtime the library's earlier tests already use
    import bench
    W = bench.WORKLOADS[name]
    L = bench.bedgen_lib()
    gens, inputs = [], []
    try:
        for (seed, mode), n, kind, pin in zip(W["gen"], W["rows"], W["kinds"], REF[name]["inputs"]):
            p, nb, rows = bench.gen(L, n, seed, (1 << 64) - 1, mode)
            gens.append(p)
            assert (rows, nb) == (pin["rows"], pin["bytes"]), (name, seed)  # the reference's inputs
            inputs.append(((p.value, nb, False), kind))
        s = eng.load(inputs)
    finally:
        for p in gens:
            L.bedgen_free(p)
    try:
        r = bench.run_op(eng, name, s)
        try:
            r.format()
            text = r.text()
        finally:
            r.free()
    finally:
        s.free()
    want = REF[name]["output"]
    got = {"rows": text.count(b"\n"), "bytes": len(text), "sha16": hashlib.sha256(text).hexdigest()[:16]}
    assert got == want, name
