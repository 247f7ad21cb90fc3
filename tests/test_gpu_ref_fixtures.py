"""The GPU drop-in binaries against the genuine reference's own output.

Every case of tests/golden/ref_*.json.gz (BEDOPS v2.4.26 built by oracle/build_ref.sh; inputs,
argv, stdout, stderr and exit status recorded by tests/golden/make_ref_fixtures.py) is re-run
through bedops_amd/bin/{bedops,bedmap,closest-features,sort-bed} — the HIP path through the
C-ABI — and must reproduce stdout byte for byte, the exit status, and (for --ec and the
element-operation stops) the error text.
"""
import pytest

import ref_fixtures as R

pytestmark = pytest.mark.gpu

CHUNK = 40
_SIZES = {"closest": 96, "bedmap": 313, "decimal": 124, "sortbed": 6, "ec": 112}
PARAMS = [(s, i) for s, n in _SIZES.items() for i in range(0, n, CHUNK)]


@pytest.mark.parametrize("suite,start", PARAMS, ids=[f"{s}-{i}" for s, i in PARAMS])
def test_gpu_cli_reproduces_reference(gpu_bin, suite, start):
    fx = R.load(suite)
    assert len(fx["cases"]) == _SIZES[suite]
    bad = []
    for k in range(start, min(start + CHUNK, len(fx["cases"]))):
        c = fx["cases"][k]
        d = R.compare(gpu_bin[c["tool"]], fx, c, check_stderr=(suite == "ec" or c["rc"] != 0))
        if d:
            bad.append((k, c["args"], d[:240]))
    assert not bad, bad
