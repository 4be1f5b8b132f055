import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "road-vision-system_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def pytest_sessionstart(session):
    """A fatal signal in native code writes its C stack before Python's
    faulthandler writes the Python one (rv_install_crash_handler)."""
    try:
        from rvs_amd import _lib
        _lib.load().rv_install_crash_handler()
    except Exception as e:  # the library may not be built in a CPU-only checkout
        os.write(2, f"[conftest] native crash handler not installed: {e}\n".encode())


def pytest_runtest_logstart(nodeid, location):
    """Name every test on stderr before it runs (unbuffered), so the tail of a
    run that dies in native code says which test it died in, even under -q."""
    os.write(2, f"\n[test start] {nodeid}\n".encode())


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def road_frame(H, W, seed=0):
    """Synthetic low-contrast road-like BGR frame."""
    rng = np.random.default_rng(seed)
    y = np.linspace(60, 170, H, dtype=np.float32)[:, None, None]
    img = np.broadcast_to(y, (H, W, 3)).astype(np.float32).copy()
    img += rng.normal(0, 3, size=(1, 1, 3)).astype(np.float32) * 4
    for _ in range(int(rng.integers(24, 49))):
        h = int(rng.integers(max(2, H // 40), max(3, H // 6)))
        w = int(rng.integers(max(2, W // 40), max(3, W // 5)))
        y0 = int(rng.integers(0, max(1, H - h)))
        x0 = int(rng.integers(0, max(1, W - w)))
        img[y0:y0 + h, x0:x0 + w] += rng.uniform(-40, 40, size=3).astype(np.float32)
    img += rng.normal(0, 6, size=img.shape).astype(np.float32)
    img = np.clip(img, 0, 255).astype(np.uint8)
    n_sp = int(0.005 * H * W)
    ys = rng.integers(0, H, n_sp)
    xs = rng.integers(0, W, n_sp)
    img[ys, xs] = rng.choice([0, 255], size=(n_sp, 1)).astype(np.uint8)
    return img
