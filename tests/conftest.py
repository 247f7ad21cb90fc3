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


def _lib_fresh():
    """the in-tree libbedgpu.so is newer than every source it is built from (the objects are
    not shipped to the GPU box: make would rebuild the whole library there, ~100 s)"""
    import glob
    lib = os.path.join(ROOT, "bedops_amd", "lib", "libbedgpu.so")
    if not os.path.exists(lib):
        return False
    srcs = glob.glob(os.path.join(ROOT, "bedops_amd", "csrc", "*")) + [os.path.join(ROOT, "include", "bedgpu.h")]
    return os.path.getmtime(lib) >= max(os.path.getmtime(f) for f in srcs)


@pytest.fixture(scope="session")
def gpu_bin():
    """The drop-in front-ends (C, linked to libbedgpu.so)."""
    if _lib_fresh():
        _make("-o", "bedops_amd/lib/libbedgpu.so", "cli")  # (-o: take the library as built)
    else:
        _make("lib", "cli")
    return {"bedops": os.path.join(ROOT, "bedops_amd", "bin", "bedops"),
            "bedmap": os.path.join(ROOT, "bedops_amd", "bin", "bedmap"),
            "closest": os.path.join(ROOT, "bedops_amd", "bin", "closest-features"),
            "sortbed": os.path.join(ROOT, "bedops_amd", "bin", "sort-bed")}


@pytest.fixture(scope="session")
def bedgen():
    _make("tools")
    return os.path.join(ROOT, "tools", "build", "bedgen")
