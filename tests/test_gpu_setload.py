"""GPU parity of the BG_BED3_SET loader (k_parse_set + k_set_count/k_set_write): inputs
parsed straight to their merged sets must give byte-identical output to the row-keeping
loader (BG_BED3 + k_components) and to the oracle, including components that span many
8 KiB tiles (absorbed local components) and every error the row loader reports."""
import random
import tempfile
import zlib

import pytest

import randbed
from test_gpu_parity import run_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from bedops_amd import Engine
    e = Engine(0)
    yield e
    e.close()


MODES = [("-m", []), ("-i", []), ("-d", []), ("-e", ["1"]), ("-n", ["30%"]), ("-c", []),
         ("-s", []), ("-w", ["7"])]


def _texts(rng, nfiles, n, maxlen, span, chroms=randbed.CHROMS):
    out = []
    for f in range(nfiles):
        rs = randbed.rows(rng, n, chroms=chroms, span=span, maxlen=maxlen)
        out.append(randbed.text(rs, rest="cols" if f == 0 else None, rng=rng).encode())
    return out


def _run(eng, mode, extra, texts, set_load):
    kw = {}
    if mode in ("-e", "-n"):
        kw["spec"] = extra[0]
    if mode == "-w":
        kw["chop"] = (int(extra[0]), 0, False)
    return eng.bedops(mode, texts, set_load=set_load, **kw)


@pytest.mark.parametrize("mode,extra", MODES)
@pytest.mark.parametrize("shape", ["sparse", "dense", "long"])
def test_set_load_matches_rows_and_oracle(eng, oracle_bin, mode, extra, shape):
    """tens of tiles per file; 'long' rows reach across many tiles so that whole tiles
    of local components are absorbed by the running max of earlier tiles"""
    rng = random.Random(zlib.crc32(repr((mode, shape)).encode()))
    n, maxlen, span = {"sparse": (6000, 20, 4_000_000), "dense": (20000, 200, 300_000),
                       "long": (20000, 30000, 2_000_000)}[shape]
    texts = _texts(rng, 2 if mode != "-s" else 3, n, maxlen, span)
    if mode not in ("-e", "-n"):
        texts[0] = randbed.text(randbed.rows(random.Random(5), n, span=span, maxlen=maxlen)).encode()
    with tempfile.TemporaryDirectory() as td:
        want = run_oracle(oracle_bin["bedops"], [mode] + extra, texts, td)
    got_set = _run(eng, mode, extra, texts, True)
    got_rows = _run(eng, mode, extra, texts, False)
    assert got_rows == want
    assert got_set == want


def test_one_row_covers_everything(eng, oracle_bin):
    """the first row spans the whole chromosome: every later tile is absorbed"""
    rng = random.Random(3)
    rs = [("chr1", 0, 900_000_000)] + randbed.rows(rng, 60000, chroms=["chr1"], span=800_000_000,
                                                    maxlen=50)
    rs.sort(key=lambda r: (r[1], r[2]))
    a = randbed.text(rs).encode()
    b = randbed.text(randbed.rows(rng, 5000, chroms=["chr1", "chr2"], span=10**9, maxlen=80)).encode()
    for mode in ("-m", "-i", "-d", "-c"):
        with tempfile.TemporaryDirectory() as td:
            want = run_oracle(oracle_bin["bedops"], [mode], [a, b], td)
        assert eng.bedops(mode, [a, b]) == want, mode
        assert eng.bedops(mode, [a, b]) == eng.bedops(mode, [a, b], set_load=False), mode


def test_set_load_edge_texts(eng, oracle_bin):
    """empty files, a single line, no final newline, odd whitespace (byte path)"""
    cases = [b"", b"chr1\t1\t5\n", b"chr1\t1\t5", b"chr1 1 5\nchr1\t3  9 x y\n",
             b"  chr1\t10\t20\n" * 3, b"chr1\t5\t5\nchr1\t5\t10\n",
             b"chrA_very_long_chromosome_name_0123456789\t5\t10\n" * 2000]
    for a in cases:
        for b in cases[:3]:
            for mode in ("-m", "-d", "-c"):
                with tempfile.TemporaryDirectory() as td:
                    want = run_oracle(oracle_bin["bedops"], [mode], [a, b], td)
                assert eng.bedops(mode, [a, b]) == want, (mode, a[:40], b[:40])


def _err(eng, text, set_load):
    from bedops_amd import BedgpuError
    with pytest.raises(BedgpuError) as ei:
        eng.bedops("-m", [text], set_load=set_load)
    return ei.value.code, ei.value.msg


@pytest.mark.parametrize("where", ["in_tile", "tile_boundary", "far"])
def test_set_load_unsorted_same_error(eng, where):
    rs = randbed.rows(random.Random(11), 30000, chroms=["chr1"], span=10**7, maxlen=40)
    lines = randbed.text(rs).encode().split(b"\n")
    k = {"in_tile": 100, "tile_boundary": None, "far": 25000}[where]
    if k is None:  # the first line that starts in the second 8 KiB tile
        pos, k = 0, 0
        while pos + len(lines[k]) + 1 <= 8192:
            pos += len(lines[k]) + 1
            k += 1
        k += 1
    lines[k] = b"chr1\t0\t1"
    text = b"\n".join(lines)
    assert _err(eng, text, True) == _err(eng, text, False)


@pytest.mark.parametrize("bad", [b"chr1\t10\t5\n", b"chr1\t5\n", b"chr1\tx\t5\n",
                                 b"chr1\t1\t1000000000000\n"])
def test_set_load_bad_line_same_error(eng, bad):
    # (a blank line is no error: test_gpu_parity.py::test_blank_lines_are_skipped_like_fscanf)
    rs = randbed.rows(random.Random(12), 3000, chroms=["chr1"], span=10**6, maxlen=40)
    lines = randbed.text(rs).encode().splitlines(keepends=True)
    text = b"".join(lines[:1500]) + bad + b"".join(lines[1500:])
    assert _err(eng, text, True) == _err(eng, text, False)


def test_set_tables_refuse_row_operations(eng):
    from bedops_amd import BedgpuError
    from bedops_amd.engine import BED3_SET
    a = randbed.text(randbed.rows(random.Random(1), 100)).encode()
    s = eng.load([(a, BED3_SET), (a, BED3_SET)])
    try:
        for call in (lambda: eng.op("-p", s, [0, 1]), lambda: eng.op("-u", s, [0, 1]),
                     lambda: eng.map_op(s, ["count"], 0, 1), lambda: eng.closest_op(s, 0, 1),
                     lambda: eng.op("-e", s, [0, 1], "1"), lambda: s.restrict_chrom("chr1")):
            with pytest.raises(BedgpuError) as ei:
                call()
            assert ei.value.code == -6
        assert s.rows(0) == 100
    finally:
        s.free()


def test_set_load_staging_overflow_falls_back(eng, oracle_bin):
    """> 512 disjoint rows in one 8 KiB tile (rows ~15 bytes) overflow the tile's staging
    slots; the load is redone with row columns and the output stays exact"""
    a = "".join(f"c\t{3 * i}\t{3 * i + 1}\n" for i in range(30000)).encode()
    b = "".join(f"c\t{5 * i}\t{5 * i + 3}\n" for i in range(18000)).encode()
    for mode in ("-m", "-i", "-d"):
        with tempfile.TemporaryDirectory() as td:
            want = run_oracle(oracle_bin["bedops"], [mode], [a, b], td)
        assert eng.bedops(mode, [a, b]) == want, mode


def test_set_load_coordinates_past_32_bits(eng, oracle_bin):
    """one-chromosome tiles scan 32-bit coordinates; an end >= 2^32 - 2 makes the loader
    redo the input with row columns, multi-chromosome tiles use 64-bit keys throughout"""
    rng = random.Random(21)
    big = 2**32 - 40
    rs = sorted((c, big + rng.randrange(200), 0) for c in ["chr1", "chr2"] for _ in range(3000))
    rs = [(c, s, s + rng.randint(1, 60)) for c, s, _ in rs]
    rs.sort(key=lambda r: (r[0], r[1], r[2]))
    a = randbed.text(rs).encode()
    b = randbed.text(randbed.rows(rng, 4000, chroms=["chr1", "chr2"], span=2**33, maxlen=10**6)).encode()
    for mode in ("-m", "-i", "-d"):
        with tempfile.TemporaryDirectory() as td:
            want = run_oracle(oracle_bin["bedops"], [mode], [a, b], td)
        assert eng.bedops(mode, [a, b], set_load=False) == want, mode  # (printing >= 2^32)
        assert eng.bedops(mode, [a, b]) == want, mode


def test_chrom_spans_of_set_results(eng):
    """the per-chromosome byte spans the multi-GPU gather uses, on set-loaded results"""
    rng = random.Random(31)
    chroms = ["chr1", "chr10", "chr2", "chr3", "chrX"]
    a = randbed.text(randbed.rows(rng, 20000, chroms=chroms[:4], span=10**6, maxlen=300)).encode()
    b = randbed.text(randbed.rows(rng, 20000, chroms=chroms[1:], span=10**6, maxlen=300)).encode()
    from bedops_amd.engine import BED3_SET
    s = eng.load([(a, BED3_SET), (b, BED3_SET)])
    try:
        names = s.chroms()
        for mode in ("-i", "-m", "-d"):
            r = eng.op(mode, s, [0, 1])
            txt = r.text()
            sp = r.chrom_spans(len(names))
            assert sp[-1] == len(txt)
            for g, nm in enumerate(names):
                part = txt[sp[g]:sp[g + 1]]
                want = b"".join(ln + b"\n" for ln in txt.split(b"\n") if ln.split(b"\t")[0] == nm.encode())
                assert part == want, (mode, nm)
            r.free()
    finally:
        s.free()


def _outcome(eng, texts, set_load):
    from bedops_amd import BedgpuError
    try:
        return ("ok", eng.bedops("-m", texts, set_load=set_load))
    except BedgpuError as e:
        return ("err", e.code, e.msg)


@pytest.mark.parametrize("where", ["token", "sep1", "start", "sep2", "end", "after_end"])
def test_set_load_every_byte(eng, where):
    """every byte value at each position of one line inside a long sorted file: the set
    loader's byte classes (whitespace, '\\n', digits; k_parse_set_v's bitop3/dot-product
    SWAR) must agree with the row loader's, whether the line is accepted or refused"""
    rs = randbed.rows(random.Random(21), 20000, chroms=["chr1"], span=10**7, maxlen=40)
    lines = randbed.text(rs).encode().splitlines(keepends=True)
    k = 9000  # far inside the file: the sub-tile takes the unguarded load path
    head, tail = b"".join(lines[:k]), b"".join(lines[k + 1:])
    c, s, e = lines[k].rstrip(b"\n").split(b"\t")
    for b in range(256):
        x = bytes([b])
        if b == 10:
            continue
        line = {"token": c[:2] + x + c[2:] + b"\t" + s + b"\t" + e,
                "sep1": c + x + s + b"\t" + e,
                "start": c + b"\t" + s[:1] + x + s[1:] + b"\t" + e,
                "sep2": c + b"\t" + s + x + e,
                "end": c + b"\t" + s + b"\t" + e[:1] + x + e[1:],
                "after_end": c + b"\t" + s + b"\t" + e + x + b"rest"}[where]
        text = head + line + b"\n" + tail
        assert _outcome(eng, [text], True) == _outcome(eng, [text], False), (where, b)


@pytest.mark.parametrize("mode,extra", MODES)
def test_long_rows_across_subtiles_equal_oracle(eng, oracle_bin, mode, extra):
    """long rows of the last file reach across hundreds of 4 KiB sub-tiles, so whole sub-tiles
    are absorbed by the running max of earlier ones (k_set_count) and components continue
    across them (k_set_write), with the earlier inputs' merge passes on the side stream"""
    rng = random.Random(zlib.crc32(repr(("split", mode)).encode()))
    n = 20000
    texts = _texts(rng, 2 if mode != "-s" else 3, n, 200, 300_000)
    long_rows = randbed.rows(rng, n, chroms=["chr1", "chr2"], span=2_000_000, maxlen=30000)
    long_rows.append(("chr1", 10, 1_500_000))  # one row over half the last file's chr1
    long_rows.sort(key=lambda r: (r[0], r[1], r[2]))
    texts[-1] = randbed.text(long_rows).encode()
    with tempfile.TemporaryDirectory() as td:
        want = run_oracle(oracle_bin["bedops"], [mode] + extra, texts, td)
    assert _run(eng, mode, extra, texts, True) == want
