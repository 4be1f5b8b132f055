"""Synthetic device-side road frames: vertical luminance
gradient 60->170, 24-48 drifting vehicle rectangles (+-40 around the local
mean), Gaussian noise sigma 6, 0.5 % salt-and-pepper rain.  Frame f of
stream s uses seed 1000*s + f for its noise; rectangles drift 2-6 px/frame so
SORT sees persistent tracks.  Used by bench.py (inputs resident in HBM before
the timed region)."""
from __future__ import annotations

import numpy as np
import torch


def road_frames(n_streams: int, n_frames: int, H: int = 1080, W: int = 1920, device="cuda",
                stream_offset: int = 0) -> torch.Tensor:
    """(n_frames, n_streams, H, W, 3) uint8 on the device."""
    dev = torch.device(device)
    out = torch.empty((n_frames, n_streams, H, W, 3), dtype=torch.uint8, device=dev)
    grad = torch.linspace(60, 170, H, device=dev).view(1, H, 1, 1)
    g = torch.Generator(device=dev)
    for s in range(n_streams):
        sid = s + stream_offset
        rng = np.random.default_rng(1000 * sid)
        tint = torch.tensor(rng.normal(0, 12, 3), dtype=torch.float32, device=dev).view(1, 1, 1, 3)
        nrect = int(rng.integers(24, 49))
        rh = rng.integers(H // 40, H // 6, nrect)
        rw = rng.integers(W // 40, W // 5, nrect)
        ry = rng.integers(0, H - rh)
        rx = rng.integers(0, W - rw)
        col = rng.uniform(-40, 40, (nrect, 3))
        vx = rng.uniform(2, 6, nrect) * rng.choice([-1, 1], nrect)
        vy = rng.uniform(-2, 2, nrect)
        for f in range(n_frames):
            img = (grad + tint).expand(1, H, W, 3).clone()
            for i in range(nrect):
                y0 = int(ry[i] + vy[i] * f) % (H - rh[i])
                x0 = int(rx[i] + vx[i] * f) % (W - rw[i])
                img[0, y0:y0 + rh[i], x0:x0 + rw[i]] += torch.tensor(col[i], dtype=torch.float32,
                                                                     device=dev)
            g.manual_seed(1000 * sid + f)
            img += torch.randn(img.shape, generator=g, device=dev) * 6
            sp = torch.rand((1, H, W, 1), generator=g, device=dev)
            img = torch.where(sp < 0.0025, torch.zeros_like(img), img)
            img = torch.where(sp > 0.9975, torch.full_like(img, 255.0), img)
            out[f, s] = img.clamp_(0, 255).to(torch.uint8)[0]
    return out
