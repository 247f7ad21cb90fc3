"""CPU checks of the drop-in boundary: the C-ABI library builds for gfx950, loads, and
exports every entry point include/bedgpu.h declares; the front-ends parse argv and
report usage errors like the reference without touching a GPU."""
import ctypes
import os
import re
import subprocess

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "bedgpu.h")).read()
    return sorted(set(re.findall(r"\b(bg_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(gpu_bin):
    from bedops_amd.engine import SYMBOLS, lib_path
    lib = ctypes.CDLL(lib_path())
    declared = _declared()
    assert declared, "no declarations parsed"
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(SYMBOLS) == declared


def test_library_contains_gfx950_code(gpu_bin):
    from bedops_amd.engine import lib_path
    data = open(lib_path(), "rb").read()
    assert b"gfx950" in data


def test_cli_usage_errors_without_gpu(gpu_bin, tmp_path):
    bed = tmp_path / "a.bed"
    bed.write_text("chr1\t1\t2\n")
    r = subprocess.run([gpu_bin["bedops"], "--intersect", str(bed)], stderr=subprocess.PIPE,
                       stdout=subprocess.PIPE)
    assert r.returncode == 1
    assert r.stderr.decode().startswith("May use bedops --help for more help.\n\nError: Bad Input\n")
    assert "Not enough files" in r.stderr.decode()
    r = subprocess.run([gpu_bin["bedops"], "-x", str(bed)], stderr=subprocess.PIPE)
    assert r.returncode == 1 and "Unknown operation: -x" in r.stderr.decode()
    r = subprocess.run([gpu_bin["bedops"], "-m", str(tmp_path / "missing.bed")], stderr=subprocess.PIPE)
    assert r.returncode == 1 and "Cannot find" in r.stderr.decode()
    r = subprocess.run([gpu_bin["bedops"], "--version"], stdout=subprocess.PIPE)
    assert r.returncode == 0 and b"2.4.26" in r.stdout
    r = subprocess.run([gpu_bin["bedmap"], "--count", "--bogus", str(bed), str(bed)], stderr=subprocess.PIPE)
    assert r.returncode == 1


def test_python_mirror_fails_loudly_without_library(monkeypatch):
    import bedops_amd.engine as E
    monkeypatch.setattr(E, "_LIB", None)
    monkeypatch.setattr(E, "lib_path", lambda: "/nonexistent/libbedgpu.so")
    try:
        E.load_library()
    except E.BedgpuError as e:
        assert "not built" in str(e)
    else:
        raise AssertionError("expected BedgpuError")


def test_overlap_spec_parsing():
    from bedops_amd.engine import parse_overlap_spec
    assert parse_overlap_spec(None) == (1.0, 1)
    assert parse_overlap_spec("50%") == (0.5, 1)
    assert parse_overlap_spec("0%") == (1.0, 0)
    assert parse_overlap_spec("3") == (3.0, 0)
    assert parse_overlap_spec("-5") == (5.0, 0)
