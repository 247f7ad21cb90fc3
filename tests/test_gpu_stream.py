"""The one-GPU chromosome-group pipeline of the front-ends (bedops_amd/cli/cli_stream.h).

With stdout a regular file and large enough inputs (BEDGPU_STREAM_MIN, lowered to 0 here),
bedops / bedmap / closest-features cut their inputs at chromosome boundaries into groups,
load -> operate -> format each group on the GPU and write group g while group g+1 is read
(bg_writer). The output must be byte-identical to the oracle (and so to the whole-file
path); an error or refusal in any group must leave exactly what the whole-file path leaves
(output truncated back, the whole-file run's message and status).
"""
import os
import random
import subprocess
import zlib

import pytest

import randbed

pytestmark = pytest.mark.gpu

CHROMS = ["chr1", "chr10", "chr11", "chr2", "chr20", "chr3", "chrM", "chrX", "chrY"]
MODES = [["-m"], ["-i"], ["-d"], ["-e", "1"], ["-n", "30%"], ["-c"], ["-c", "-L"], ["-w", "7"],
         ["-s"], ["-p"], ["-u"]]


def _run(exe, args, out_path, groups, stream=True, prefix=b""):
    env = dict(os.environ, BEDGPU_STATS="1", BEDGPU_STREAM_MIN="0", BEDGPU_STREAM_GROUPS=str(groups),
               BEDGPU_STREAM="1" if stream else "0")
    env.pop("BEDGPU_DEVICES", None)
    with open(out_path, "wb") as fo:
        fo.write(prefix)
        fo.flush()
        r = subprocess.run([exe, *args], stdout=fo, stderr=subprocess.PIPE, env=env, timeout=120)
    with open(out_path, "rb") as f:
        return r.returncode, f.read(), r.stderr.decode(errors="replace")


def _streamed(err):
    return "bedgpu host  group1" in err and "pipeline stopped" not in err


@pytest.mark.parametrize("mode", MODES)
def test_bedops_groups_equal_oracle(gpu_bin, oracle_bin, tmp_path, mode):
    rng = random.Random(zlib.crc32(repr(mode).encode()))
    for trial in range(3):
        files = []
        for f in range(3 if mode[0] in ("-m", "-i", "-u") else 2):
            rows = randbed.rows(rng, rng.choice([1, 600, 4000]),
                                chroms=rng.sample(CHROMS, rng.choice([1, 5, 9])),
                                span=rng.choice([500, 5000]), maxlen=rng.choice([10, 120]),
                                zero_frac=0.05 if mode[0] in ("-i", "-d", "-e", "-n") else 0.0)
            p = str(tmp_path / f"f{trial}_{f}.bed")
            randbed.write(p, randbed.text(rows, rest="cols" if f == 0 else None, rng=rng))
            files.append(p)
        want = subprocess.run([oracle_bin["bedops"], *mode, *files], stdout=subprocess.PIPE,
                              check=True).stdout
        for groups in (2, 3, 9):
            rc, got, err = _run(gpu_bin["bedops"], mode + files, str(tmp_path / "out.bed"), groups)
            assert rc == 0, err
            assert got == want, (mode, trial, groups)


@pytest.mark.parametrize("ahead", [1, 2, 5])
def test_groups_read_ahead_equal_oracle(gpu_bin, oracle_bin, tmp_path, ahead):
    """BEDGPU_STREAM_AHEAD: a copier thread copies later groups on the prefetch stream while
    earlier ones run (bg_file_image_copy after bg_copy_order, bg_copy_fence before the load):
    many small groups, so released blocks come straight back as the next groups' buffers"""
    rng = random.Random(90 + ahead)
    files = [randbed.write(str(tmp_path / f"{k}.bed"),
                           randbed.text(randbed.rows(rng, 30000, chroms=CHROMS, span=60000)))
             for k in range(2)]
    os.environ["BEDGPU_STREAM_AHEAD"] = str(ahead)
    try:
        for mode in (["-i"], ["-m"], ["-d"]):
            want = subprocess.run([oracle_bin["bedops"], *mode, *files], stdout=subprocess.PIPE,
                                  check=True).stdout
            for groups in (3, 9):
                rc, got, err = _run(gpu_bin["bedops"], mode + files, str(tmp_path / "o.bed"), groups)
                assert rc == 0 and got == want, (mode, groups, err[-2000:])
                assert _streamed(err), err
    finally:
        os.environ.pop("BEDGPU_STREAM_AHEAD", None)


@pytest.mark.parametrize("ops", [["--bp-ovr", "5", "--median", "--indicator"],
                                 ["--fraction-ref", "0.5", "--mean", "--echo-map-range"],
                                 ["--range", "20", "--count", "--min-element", "--skip-unmapped"]])
def test_bedmap_groups_read_ahead_equal_oracle(gpu_bin, oracle_bin, tmp_path, ops):
    """the bedmap cases that faulted under read-ahead in round 4 (test_bedmap_groups_equal_oracle
    ops2..ops4 with BEDGPU_STREAM_AHEAD on): a group's text is copied on the prefetch stream
    after the previous group's kernels released its blocks (bg_copy_order), and the formatter's
    write pass checks every row against its count (BG_FMT_MISMATCH) instead of trusting it"""
    rng = random.Random(zlib.crc32(repr(("ahead", ops)).encode()))
    ref = randbed.write(str(tmp_path / "r.bed"),
                        randbed.text(randbed.rows(rng, 3000, chroms=CHROMS, span=8000), rest="cols", rng=rng))
    mp = randbed.write(str(tmp_path / "m.bed"),
                       _scored(rng, randbed.rows(rng, 6000, chroms=CHROMS[:7], span=8000)))
    for ahead in (1, 2, 5):
        os.environ["BEDGPU_STREAM_AHEAD"] = str(ahead)
        try:
            for args in (ops + [ref, mp], ops + [mp]):
                want = subprocess.run([oracle_bin["bedmap"], *args], stdout=subprocess.PIPE, check=True).stdout
                for groups in (2, 5):
                    rc, got, err = _run(gpu_bin["bedmap"], args, str(tmp_path / "o.bed"), groups)
                    assert rc == 0, err[-2000:]
                    assert got == want, (args, groups, ahead)
        finally:
            os.environ.pop("BEDGPU_STREAM_AHEAD", None)


def test_bedops_groups_actually_stream(gpu_bin, oracle_bin, tmp_path):
    rng = random.Random(3)
    files = [randbed.write(str(tmp_path / f"{k}.bed"),
                           randbed.text(randbed.rows(rng, 20000, chroms=CHROMS, span=50000)))
             for k in range(2)]
    want = subprocess.run([oracle_bin["bedops"], "-i", *files], stdout=subprocess.PIPE, check=True).stdout
    rc, got, err = _run(gpu_bin["bedops"], ["-i", *files], str(tmp_path / "o.bed"), 4)
    assert rc == 0 and got == want
    assert _streamed(err), err
    # output appended after bytes already in the file (fd at a non-zero offset, not O_APPEND)
    rc, got, err = _run(gpu_bin["bedops"], ["-i", *files], str(tmp_path / "o.bed"), 4, prefix=b"head\n")
    assert rc == 0 and got == b"head\n" + want
    assert _streamed(err), err
    # below the size threshold and with BEDGPU_STREAM=0: the whole-file path, same bytes
    rc, got2, err = _run(gpu_bin["bedops"], ["-i", *files], str(tmp_path / "o.bed"), 4, stream=False)
    assert rc == 0 and got2 == want and "group1" not in err


@pytest.mark.parametrize("bad", ["chr3\t4\tx\n", "chr3\t9\t5\n", "chr20\t1\t2\n"])
def test_error_in_a_later_group_matches_whole_file(gpu_bin, tmp_path, bad):
    """a malformed / out-of-range / unsorted line in a later group: the groups written before
    it are truncated away and the whole-file path reports the error (same status, message,
    line number, empty output)"""
    rng = random.Random(11)
    rows = randbed.rows(rng, 3000, chroms=["chr1", "chr2", "chr3", "chrX"], span=20000)
    t = randbed.text(rows)
    lines = t.splitlines(keepends=True)
    k = next(i for i, ln in enumerate(lines) if ln.startswith("chr3\t"))
    lines.insert(k + 5, bad)
    a = randbed.write(str(tmp_path / "a.bed"), "".join(lines))
    b = randbed.write(str(tmp_path / "b.bed"), randbed.text(randbed.rows(rng, 2000, chroms=["chr1", "chr3"])))
    for groups in (2, 4):
        want = _run(gpu_bin["bedops"], ["-i", a, b], str(tmp_path / "w.bed"), groups, stream=False,
                    prefix=b"keep\n")
        got = _run(gpu_bin["bedops"], ["-i", a, b], str(tmp_path / "g.bed"), groups, prefix=b"keep\n")
        assert want[0] != 0
        assert got[0] == want[0] and got[1] == want[1] == b"keep\n"
        assert got[2].splitlines()[-1] == want[2].splitlines()[-1]


def _scored(rng, rows, decimal_from=None):
    out = []
    for i, (c, s, e) in enumerate(rows):
        sc = rng.randint(0, 50)
        if decimal_from and c >= decimal_from:
            sc = f"{sc}.{rng.randint(0, 99):02d}"
        out.append(f"{c}\t{s}\t{e}\tid{i}\t{sc}\n")
    return "".join(out)


@pytest.mark.parametrize("ops", [["--count", "--mean"], ["--echo", "--sum", "--max", "--echo-map-id"],
                                 ["--bp-ovr", "5", "--median", "--indicator"],
                                 ["--fraction-ref", "0.5", "--mean", "--echo-map-range"],
                                 ["--range", "20", "--count", "--min-element", "--skip-unmapped"]])
def test_bedmap_groups_equal_oracle(gpu_bin, oracle_bin, tmp_path, ops):
    rng = random.Random(zlib.crc32(repr(ops).encode()))
    ref = randbed.write(str(tmp_path / "r.bed"),
                        randbed.text(randbed.rows(rng, 3000, chroms=CHROMS, span=8000), rest="cols", rng=rng))
    mp = randbed.write(str(tmp_path / "m.bed"),
                       _scored(rng, randbed.rows(rng, 6000, chroms=CHROMS[:7], span=8000)))
    for args in (ops + [ref, mp], ops + [mp]):  # two files; single-file mode
        want = subprocess.run([oracle_bin["bedmap"], *args], stdout=subprocess.PIPE, check=True).stdout
        for groups in (2, 5):
            rc, got, err = _run(gpu_bin["bedmap"], args, str(tmp_path / "o.bed"), groups)
            assert rc == 0, err
            assert got == want, (args, groups)
            if ops == ["--count", "--mean"]:  # others may meet address-ordered ties (refused:
                assert _streamed(err), err    # one heap history per file) and fall back


def test_bedmap_decimal_scores_in_a_later_group_fall_back(gpu_bin, oracle_bin, tmp_path):
    """decimal scores sum into one double across the whole file: a group meeting them is
    refused, the output so far dropped, and the whole-file path gives the oracle's bytes"""
    rng = random.Random(21)
    ref = randbed.write(str(tmp_path / "r.bed"), randbed.text(randbed.rows(rng, 3000, chroms=CHROMS, span=8000)))
    mp = randbed.write(str(tmp_path / "m.bed"),
                       _scored(rng, randbed.rows(rng, 6000, chroms=CHROMS, span=8000), decimal_from="chrX"))
    want = subprocess.run([oracle_bin["bedmap"], "--mean", "--sum", ref, mp], stdout=subprocess.PIPE,
                          check=True).stdout
    rc, got, err = _run(gpu_bin["bedmap"], ["--mean", "--sum", ref, mp], str(tmp_path / "o.bed"), 4)
    assert rc == 0 and got == want, err
    assert "pipeline stopped" in err


@pytest.mark.parametrize("opts", [["--closest"], [], ["--dist"], ["--closest", "--dist", "--no-ref"],
                                  ["--no-overlaps", "--closest", "--delim", "|"]])
def test_closest_groups_equal_oracle(gpu_bin, oracle_bin, tmp_path, opts):
    rng = random.Random(zlib.crc32(repr(opts).encode()))
    q = randbed.write(str(tmp_path / "q.bed"),
                      randbed.text(randbed.rows(rng, 2000, chroms=CHROMS[2:], span=30000), rest="cols", rng=rng))
    r = randbed.write(str(tmp_path / "r.bed"),
                      randbed.text(randbed.rows(rng, 5000, chroms=CHROMS[:6], span=30000), rest="cols", rng=rng))
    want = subprocess.run([oracle_bin["closest"], *opts, q, r], stdout=subprocess.PIPE, check=True).stdout
    for groups in (2, 7):
        rc, got, err = _run(gpu_bin["closest"], opts + [q, r], str(tmp_path / "o.bed"), groups)
        assert rc == 0, err
        assert got == want, (opts, groups)
        assert _streamed(err), err


def test_detached_teardown_status_and_output(gpu_bin, oracle_bin, tmp_path):
    """cli_detach: the front process returns once the worker's output is complete, with the
    worker's status; stdout/stderr pipes see EOF; failures are mirrored"""
    rng = random.Random(8)
    a = randbed.write(str(tmp_path / "a.bed"), randbed.text(randbed.rows(rng, 5000, chroms=CHROMS)))
    b = randbed.write(str(tmp_path / "b.bed"), randbed.text(randbed.rows(rng, 5000, chroms=CHROMS)))
    want = subprocess.run([oracle_bin["bedops"], "-u", a, b], stdout=subprocess.PIPE, check=True).stdout
    for det in ("1", "0"):
        env = dict(os.environ, BEDGPU_DETACH=det)
        r = subprocess.run([gpu_bin["bedops"], "-u", a, b], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           env=env, timeout=120)
        assert r.returncode == 0 and r.stdout == want, r.stderr
        with open(a, "rb") as fi:  # stdin read by the worker
            r = subprocess.run([gpu_bin["bedops"], "-u", "-", b], stdin=fi, stdout=subprocess.PIPE,
                               stderr=subprocess.PIPE, env=env, timeout=120)
        assert r.returncode == 0 and r.stdout == want, r.stderr
        bad = randbed.write(str(tmp_path / "bad.bed"), "chr1\t5\t1\n")
        r = subprocess.run([gpu_bin["bedops"], "-u", bad, b], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           env=env, timeout=120)
        assert r.returncode == 1 and b"Error" in r.stderr and r.stdout == b""


def _run_pipe(exe, args, groups, stream=True):
    env = dict(os.environ, BEDGPU_STATS="1", BEDGPU_STREAM_MIN="0", BEDGPU_STREAM_GROUPS=str(groups),
               BEDGPU_STREAM="1" if stream else "0")
    env.pop("BEDGPU_DEVICES", None)
    r = subprocess.run([exe, *args], stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=120)
    return r.returncode, r.stdout, r.stderr.decode(errors="replace")


def test_groups_through_a_pipe(gpu_bin, oracle_bin, tmp_path):
    """stdout a pipe: the groups go out in order as they are done (bg_writer, 1 MiB pipe
    buffer); a refusal in a later group (decimal sums) reruns the whole file and continues the
    output after the groups already written (bg_set_output_skip): the oracle's bytes either way"""
    rng = random.Random(31)
    files = [randbed.write(str(tmp_path / f"{k}.bed"),
                           randbed.text(randbed.rows(rng, 20000, chroms=CHROMS, span=50000)))
             for k in range(2)]
    want = subprocess.run([oracle_bin["bedops"], "-i", *files], stdout=subprocess.PIPE, check=True).stdout
    for groups in (2, 5):
        rc, got, err = _run_pipe(gpu_bin["bedops"], ["-i", *files], groups)
        assert rc == 0 and got == want, err
        assert _streamed(err), err
    ref = randbed.write(str(tmp_path / "r.bed"), randbed.text(randbed.rows(rng, 3000, chroms=CHROMS, span=8000)))
    mp = randbed.write(str(tmp_path / "m.bed"),
                       _scored(rng, randbed.rows(rng, 6000, chroms=CHROMS, span=8000), decimal_from="chrX"))
    want = subprocess.run([oracle_bin["bedmap"], "--mean", "--sum", ref, mp], stdout=subprocess.PIPE,
                          check=True).stdout
    rc, got, err = _run_pipe(gpu_bin["bedmap"], ["--mean", "--sum", ref, mp], 4)
    assert rc == 0 and got == want, err
    assert "pipeline stopped" in err


def test_error_in_a_later_group_through_a_pipe(gpu_bin, tmp_path):
    """stdout a pipe and a malformed line in a later group: the groups before it are out
    already, then the whole-file path's message and exit status"""
    rng = random.Random(12)
    rows = randbed.rows(rng, 3000, chroms=["chr1", "chr2", "chr3", "chrX"], span=20000)
    lines = randbed.text(rows).splitlines(keepends=True)
    k = next(i for i, ln in enumerate(lines) if ln.startswith("chr3\t"))
    lines.insert(k + 5, "chr3\t4\tx\n")
    a = randbed.write(str(tmp_path / "a.bed"), "".join(lines))
    b = randbed.write(str(tmp_path / "b.bed"), randbed.text(randbed.rows(rng, 2000, chroms=["chr1", "chr3"])))
    want_rc, _, want_err = _run_pipe(gpu_bin["bedops"], ["-i", a, b], 4, stream=False)
    rc, got, err = _run_pipe(gpu_bin["bedops"], ["-i", a, b], 4)
    assert want_rc != 0 and rc == want_rc
    assert err.splitlines()[-1] == want_err.splitlines()[-1]
