"""CPU test of the loader's branch-free field extraction (bedops_amd/csrc/bg_parse.h):
the same header the GPU kernel uses, compiled with g++, against a plain restatement of
the accepted line grammar. Lines the SWAR path cannot decide must report "slow" (the
kernel then runs the byte-by-byte grammar), never a wrong value."""
import os
import random
import re
import subprocess

from conftest import ROOT

WS = " \t\r\v\f"


def ref_parse(line):
    """[ws] chrom ws+ digits ws+ digits rest -> (a0, a1, start, end, rest) or None"""
    m = re.match(r"^([ \t\r\v\f]*)([^ \t\r\v\f]+)[ \t\r\v\f]+([0-9]+)[ \t\r\v\f]+([0-9]+)", line)
    if not m:
        return None
    a0 = len(m.group(1))
    a1 = a0 + len(m.group(2))
    return a0, a1, int(m.group(3)), int(m.group(4)), m.end()


def test_swar_fields_match_grammar(tmp_path):
    exe = str(tmp_path / "ph")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe,
                    os.path.join(ROOT, "tests", "cpu", "parse_helpers_main.cpp")], check=True)
    rng = random.Random(3)
    lines = ["chr1\t5\t10", "chr10\t0\t1\tfoo", "1 2 3", "  chrX\t123456789012\t999999999999",
             "chr1\t5\t", "chr1\t5x\t10", "chr1\t+5\t10", "", "   ", "chr1\t0005\t00010\t\r",
             "chr1\t5\t10\x80\xff", "c\x00r\t1\t2", "chr22_KI270731v1_random\t1\t2",
             "chrUn_very_long_contig_name_abcdefghij\t1\t2", "chr1\t1234567890123456\t1"]
    for _ in range(3000):
        name = rng.choice(["chr1", "chr10", "chrX", "1", "chrUn_gl000220", "c" * rng.randint(1, 30)])
        sep = lambda: "".join(rng.choice(WS) for _ in range(rng.choice([1, 1, 1, 2, 3])))  # noqa: E731
        s = rng.randint(0, 10 ** rng.randint(1, 12) - 1)
        e = s + rng.randint(0, 10 ** rng.randint(1, 4))
        sd = str(s).zfill(rng.choice([0, 0, 0, 5, 14]))
        rest = rng.choice(["", "", "\tid\t5\t+", " x", "\r", "\tname" * 5])
        lead = rng.choice(["", "", " ", "\t\t"])
        lines.append(f"{lead}{name}{sep()}{sd}{sep()}{e}{rest}")
    p = subprocess.run([exe], input="\n".join(lines).encode("latin-1") + b"\n",
                       stdout=subprocess.PIPE, check=True)
    outs = p.stdout.decode().splitlines()
    assert len(outs) == len(lines)
    nfast = nfast_ws = 0
    for ln, full in zip(lines, outs):
        r = ref_parse(ln)
        # the whitespace-only split: fast only where the grammar gives the same fields and
        # the end digits run to whitespace or the line end
        ws, out = full.split(" ", 1)[1], ""
        if ws.startswith("fast "):
            f = ws.split()
            _, a0, a1, s, e, rest = f[:6]
            out = " ".join(f[6:])
            nfast_ws += 1
            assert r is not None, ln
            assert (int(a0), int(a1), int(s), int(e), int(rest)) == r, (ln, ws, r)
            assert rest == str(len(ln)) or ln[int(rest)] in WS, ln
        else:
            out = ws.split(" ", 1)[1]
            if ws.startswith("blank "):
                assert ln.strip(WS) == "", ln
        if out == "blank":
            assert ln.strip(WS) == "", ln
            continue
        if out == "slow":
            continue
        nfast += 1
        _, a0, a1, s, e, rest = out.split()
        assert r is not None, ln
        assert (int(a0), int(a1), int(s), int(e), int(rest)) == r, (ln, out, r)
    assert nfast > 2000  # the common shapes take the fast path
    assert nfast_ws > 1800  # (the old count includes 13-16 digit numbers, which the kernel sends to the byte path too)
