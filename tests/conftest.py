import os
import sys

import pytest

# PyTorch bundles its own HIP runtime (ROCm 7.0) while libvxslam.so links the system one (7.2);
# both carry the soname libamdhip64.so.7, so whichever a process loads first serves both.  torch only
# initialises on its own copy: load it before any test loads libvxslam (a full-suite run does this
# anyway when collecting the modules that import torch; a narrower selection might not).
# (not under the ASan run of tests/test_sanitizers.py, which preloads libasan: the CPU tests it runs
# need no torch, and torch's ROCm libraries are not built for a preloaded sanitizer runtime)
if not os.environ.get("VX_SANITIZE"):
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover
        torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "visionx-slam_amd", "python"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")
    config.addinivalue_line("markers", "slow: larger-than-default sizes")
    config.addinivalue_line("markers", "sanitizer: runs the CPU suite under ASan/UBSan (not inside itself)")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle

    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def ctx():
    import vxslam

    c = vxslam.Context(0)
    yield c
    c.close()


@pytest.fixture
def slot_sums(monkeypatch):
    """The fused LocalBA with its per-keyframe partial slots (VX_BA_ATOMIC_ROWS=0, read at plan
    build) instead of the default row sums by float atomics: every run bitwise the same, for the
    tests that compare two runs (or two plan builds) bit for bit."""
    monkeypatch.setenv("VX_BA_ATOMIC_ROWS", "0")
