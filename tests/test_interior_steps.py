"""CPU: the march kernel's interior_steps bound (vr_kernels.hip) -- steps 1..K of a ray stay
strictly inside (0, 1)^3 under float32 accumulation p += fl(d * step), so the kernel may skip
the bounds and default-slab tests there.  Restated here in double exactly as the kernel
computes it, and checked against float32 marching of random rays: entry on every face, grazing
directions, tiny and large steps."""
import math

import numpy as np


def interior_steps(p, d, step, nsteps):
    delta = 2.0 ** -24
    K = float(nsteps - 1)
    for a in range(3):
        s = float(np.float32(np.float32(d[a]) * np.float32(step)))
        q = float(p[a])
        for A, B in ((q, s - delta), (1.0 - q, -(s + delta))):
            if not (A + B > 0.0):
                return 0
            if B < 0.0:
                K = min(K, math.floor(A / -B) - 1.0)
    return int(K) if K > 0.0 else 0


def test_interior_steps_never_leave_the_open_cube():
    rng = np.random.default_rng(5)
    checked = 0
    for trial in range(3000):
        # entry point on a random face (that coordinate exactly 0 or 1), direction inward
        p = rng.random(3).astype(np.float32)
        ax = rng.integers(3)
        side = rng.integers(2)
        p[ax] = np.float32(side)
        d = rng.normal(size=3)
        if trial % 5 == 0:  # grazing: almost parallel to the entry face
            d[ax] = 1e-4 * abs(d[ax])
        d[ax] = abs(d[ax]) if side == 0 else -abs(d[ax])
        d = (d / np.linalg.norm(d)).astype(np.float32)
        step = np.float32([0.005, 0.0007, 0.05, 0.3][trial % 4])
        nsteps = int(np.float32(1.8) / step)
        K = interior_steps(p, d, step, nsteps)
        q = p.copy()
        inc = (d * step).astype(np.float32)  # fl(d * step), as the kernel
        for k in range(1, K + 1):
            q = (q + inc).astype(np.float32)
            assert np.all(q > 0) and np.all(q < 1), (trial, k, K, q)
        checked += K
    assert checked > 100000  # the bound is not vacuous
