"""CPU test of the formatter's exact decimal path (bedops_amd/csrc/bg_decfmt.h): the same
header the GPU formatter uses, compiled with g++, against glibc printf "%.*lf" / "%.*e" —
what the reference prints scores with (Formats.hpp:42-50) — on edge values (ties, 2^53..2^64,
subnormals, DBL_MAX, 1e-300) and random doubles at precisions 0..1100."""
import os
import subprocess

from conftest import ROOT


def test_exact_decimal_matches_glibc(tmp_path):
    exe = str(tmp_path / "decfmt")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tests", "cpu", "decfmt_main.cpp")],
                   check=True)
    for seed in (1, 7):
        r = subprocess.run([exe, str(seed), "300000"], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout[-2000:]
        assert r.stdout.startswith("ok ")


def test_exact_score_conversion_matches_glibc_strtod(tmp_path):
    """bedops_amd/csrc/bg_strtod.h (k_score_big: scores past 19 significant digits or the
    128-bit exponent range) against glibc strtod — B5Rest reads scores with fscanf "%lf"
    (Bed.hpp:829-860): near-halfway strings, exact halfway points, subnormals, overflow"""
    exe = str(tmp_path / "strtod")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tests", "cpu", "strtod_main.cpp")],
                   check=True)
    for seed in (1, 9):
        r = subprocess.run([exe, str(seed), "200000"], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout[-2000:]
        assert r.stdout.startswith("ok ")
