"""Passive tracer ("food") seeding of StokesFood.py:420-436."""
from __future__ import annotations

import numpy as np


def tracer_init(squirmer_radius=0.25, center=(0.5, 0.5), density=25, L=1.0, H=1.0):
    """25x25 grid on [0.05, 0.95]^2 minus the points with |x - c| <= R (StokesFood.py:421-429)."""
    xx = np.linspace(0.05, L - 0.05, density)
    yy = np.linspace(0.05, H - 0.05, density)
    gx, gy = np.meshgrid(xx, yy)
    pts = np.vstack([gx.ravel(), gy.ravel()]).T
    d = np.linalg.norm(pts - np.asarray(center, dtype=np.float64), axis=1)
    return np.ascontiguousarray(pts[d > squirmer_radius])
