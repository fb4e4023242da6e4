import os
import sys

import pytest

# Load PyTorch (and its HIP runtime) before libbwrt.so, so that both share one
# HIP runtime (same soname) and torch streams / tensors can be passed to the
# C ABI (bench.py does the same).
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "bwidman-raytracer_amd"), os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")

# the tests force launch knobs (BWRT_BLOCK, BWRT_GREC, BWRT_SPREAD, ...): the
# library reads them only under BWRT_TUNING=1 (test_host_io checks the gate)
os.environ.setdefault("BWRT_TUNING", "1")
# a stray knob in the caller's environment would change which kernel every
# default-policy test checks: only the tests themselves set them (BWRT_LIB
# picks the library, BWRT_TUNING opens the gate).  The one deliberate way in
# is BWRT_AB_ENV="BWRT_X=1,BWRT_Y=2": tools/ab.sh's parity gate names a
# candidate's launch knobs there, and they are re-applied after the strip
# (and after every test), so the gate checks the candidate it reports on.
_KEEP = ("BWRT_LIB", "BWRT_TUNING", "BWRT_AB_ENV")


def ab_knobs(spec):
    """Parse BWRT_AB_ENV: comma-separated BWRT_*=value pairs."""
    out = {}
    for item in filter(None, (spec or "").split(",")):
        k, sep, v = item.partition("=")
        if not sep or not k.startswith("BWRT_") or k in _KEEP:
            raise ValueError(f"BWRT_AB_ENV: bad knob {item!r}")
        out[k] = v
    return out


_AB_KNOBS = ab_knobs(os.environ.get("BWRT_AB_ENV"))


def _reset_knobs():
    for k in [k for k in os.environ if k.startswith("BWRT_") and k not in _KEEP]:
        del os.environ[k]
    os.environ.update(_AB_KNOBS)


_reset_knobs()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libbwrt.so / HIP)")
    config.addinivalue_line("markers", "slow: long CPU oracle runs")


@pytest.fixture(autouse=True)
def _no_stray_knobs():
    """Knobs a test sets through monkeypatch are undone by it; this catches
    any left behind by a test that set os.environ directly."""
    yield
    _reset_knobs()


@pytest.fixture(scope="session")
def oracle():
    import oracle as O  # tests may use the oracle (checker only)
    O.build()
    return O


@pytest.fixture(scope="session")
def bwrt_lib():
    from bwrt import abi
    return abi.load()  # raises if libbwrt.so is missing: no fallback


@pytest.fixture(scope="session")
def gpu(bwrt_lib):
    from bwrt import Renderer
    if bwrt_lib.rt_device_count() <= 0:
        pytest.fail("no HIP device visible: GPU tests must run on an MI355X")
    r = Renderer(0, lib=bwrt_lib)
    yield r
    r.close()
