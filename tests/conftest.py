import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP library)")
    config.addinivalue_line("markers", "slow: large-input parity (minutes)")


def _make(*targets):
    subprocess.run(["make", "-s", "-j8", *targets], cwd=ROOT, check=True,
                   stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def oracle_bin():
    _make("oracle")
    return {"bedops": os.path.join(ROOT, "oracle", "build", "bedops_oracle"),
            "bedmap": os.path.join(ROOT, "oracle", "build", "bedmap_oracle"),
            "closest": os.path.join(ROOT, "oracle", "build", "closest_oracle"),
            "sortbed": os.path.join(ROOT, "oracle", "build", "sortbed_oracle")}


def tree_build_hash():
    """the content hash the Makefile would embed for this tree and its flags"""
    r = subprocess.run(["make", "-s", "print-hash"], cwd=ROOT, check=True, stdout=subprocess.PIPE)
    return r.stdout.decode().strip()


def lib_build_hash():
    """the build hash embedded in the in-tree libbedgpu.so (None when it is missing), read from
    the file: a library dlopen'ed once stays loaded, so a rebuilt one would not be seen"""
    import re
    lib = os.path.join(ROOT, "bedops_amd", "lib", "libbedgpu.so")
    if not os.path.exists(lib):
        return None
    with open(lib, "rb") as f:
        m = re.search(rb"bedgpu-build-hash:([0-9a-f]{32})", f.read())
    return m.group(1).decode() if m else None


def _lib_fresh():
    """the in-tree libbedgpu.so was built from exactly this tree's sources, Makefile and flags
    (content hash, not mtimes: a checkout or the copy to the GPU box resets those). Objects are
    not shipped to the GPU box, so a fresh library is taken as built there (no ~100 s rebuild)."""
    have = lib_build_hash()
    return have is not None and have == tree_build_hash()


@pytest.fixture(scope="session")
def gpu_bin():
    """The drop-in front-ends (C, linked to libbedgpu.so)."""
    if _lib_fresh():
        _make("-o", "bedops_amd/lib/libbedgpu.so", "cli")  # (-o: take the library as built)
    else:
        sys.stderr.write("conftest: libbedgpu.so is missing or was built from other sources; rebuilding\n")
        _make("lib", "cli")
        assert _lib_fresh(), "libbedgpu.so does not carry this tree's build hash after a rebuild"
    return {"bedops": os.path.join(ROOT, "bedops_amd", "bin", "bedops"),
            "bedmap": os.path.join(ROOT, "bedops_amd", "bin", "bedmap"),
            "closest": os.path.join(ROOT, "bedops_amd", "bin", "closest-features"),
            "sortbed": os.path.join(ROOT, "bedops_amd", "bin", "sort-bed")}


@pytest.fixture(scope="session")
def bedgen():
    _make("tools")
    return os.path.join(ROOT, "tools", "build", "bedgen")
