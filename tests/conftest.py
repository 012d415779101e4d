import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kd-via-fm-in-asr_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device and libkdfm.so")


import pytest  # noqa: E402


@pytest.fixture(autouse=True)
def _restore_kernel_modes():
    """Tests that switch the process-global MFMA arithmetic / deterministic-reduction modes must
    not leak them into later tests (test order changed the mode a parity test ran in)."""
    from kdfm import kernels as K
    saved = (K.get_math(), K.get_deterministic())
    yield
    K.set_math(saved[0])
    if K.get_deterministic() != saved[1]:
        K.set_deterministic(saved[1])
