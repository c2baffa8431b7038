import gzip
import json
import os
import subprocess
import sys

import pytest

try:  # torch first: its libamdhip64 must be the one libkmeranno.so binds to (same SONAME)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the CPU tests
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kmers.anno_amd")
for p in (ROOT, os.path.join(PKG, "python")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libkmeranno.so)")


@pytest.fixture(scope="session")
def native_lib():
    """libkmeranno.so, built in-tree if missing (hipcc cross-compiles without a GPU)."""
    lib = os.path.join(PKG, "build", "libkmeranno.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", PKG, "build/libkmeranno.so"], check=True)
    import kmeranno
    return kmeranno.load()


@pytest.fixture(autouse=True)
def _library_options():
    """Every test starts and ends with the library's default tuning options (tests that force a
    layout, block size or grid set them through the ABI, kma_option_set)."""
    yield
    import kmeranno
    if kmeranno._lib is not None:
        kmeranno.reset_options()


@pytest.fixture(scope="session")
def oracle_c():
    from oracle import c_oracle
    c_oracle.build()
    return c_oracle


@pytest.fixture(scope="session")
def small_gto():
    """The reference's own test fixture src/test/small.gto (committed gzipped)."""
    with gzip.open(os.path.join(GOLDEN, "small.gto.gz"), "rt") as f:
        return json.load(f)
