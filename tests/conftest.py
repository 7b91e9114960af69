"""Test configuration: paths, the `gpu` marker, shared fixtures.

`-m "not gpu"` (CPU container): oracle vs golden fixtures, host logic, the
C-ABI library loads and exports every symbol of include/ipls_agg.h, gloo
world-size-2 sharding.  `-m gpu` (MI355X): parity of the HIP path through the
C-ABI against the oracle and the golden fixtures.
"""
import json
import sys
from pathlib import Path

import numpy as np
import pytest

# torch first: its bundled HIP runtime must be the one in the process before
# anything loads libipls_agg.so (which links /opt/rocm's).  The other order --
# the library loaded, then torch imported and initialised -- leaves the
# library with "no HIP device available" (tools/jni_open_probe.py late_torch,
# profiles/r04/i/); a test module that loads the library without importing
# torch itself (test_jni.py) must not depend on an earlier module having
# imported it.
import torch  # noqa: F401,E402

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "ipls-java-api_amd"
GOLDEN = ROOT / "tests" / "golden"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) -- run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    with np.load(GOLDEN / "golden.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden_meta():
    return json.loads((GOLDEN / "golden.json").read_text())


@pytest.fixture(scope="session")
def ethmodel():
    import gzip
    raw = gzip.decompress((GOLDEN / "ethmodel.f64be.gz").read_bytes())
    return np.frombuffer(raw, dtype=">f8").astype(np.float64)


def bits(x):
    return np.ascontiguousarray(x, dtype=np.float64).view(np.uint64)


def assert_bits_equal(a, b, what=""):
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    assert a.shape == b.shape, f"{what}: shape {a.shape} != {b.shape}"
    ba, bb = bits(a), bits(b)
    # NaN payloads are not specified by Java (JLS 15.18.2); NaN must meet NaN.
    nan = np.isnan(a) & np.isnan(b)
    bad = (ba != bb) & ~nan
    if bad.any():
        i = int(np.flatnonzero(bad)[0])
        raise AssertionError(f"{what}: {int(bad.sum())} elements differ; first at {i}: "
                             f"{a[i]!r} ({ba[i]:#x}) != {b[i]!r} ({bb[i]:#x})")
