"""Ray sets shared by the oracle and GPU traversal tests (test infrastructure)."""
import numpy as np


def grazing_rays(sd, n, seed):
    """Rays that start on an axis-aligned face and run (almost) inside its plane: the
    envmap shadow rays of the city stand-in whose sampled direction lies in a wall's
    plane.  Moller-Trumbore accepts edge hits on coplanar neighbours a rounding error
    outside their exact boxes, so these pin the conservative (padded) box culling.
    Returns (rays[n, 8], last_hit[n])."""
    rng = np.random.default_rng(seed)
    V = sd.vertices.astype(np.float32)
    I = sd.triangle_indices.reshape(-1, 3)
    A, B, C = V[I[:, 0]], V[I[:, 1]], V[I[:, 2]]
    nrm = np.cross(B - A, C - A)
    ax = np.argmax(np.abs(nrm), axis=1)
    flat = np.flatnonzero((np.abs(nrm) > 0).sum(1) == 1)        # exactly axis-aligned faces
    pick = rng.choice(flat, n)
    r1, r2 = rng.random(n).astype(np.float32), rng.random(n).astype(np.float32)
    s = np.sqrt(r1)
    u, v = 1 - s, (1 - r2) * s
    o = (A[pick] + (B[pick] - A[pick]) * u[:, None] + (C[pick] - A[pick]) * v[:, None]).astype(np.float32)
    a = ax[pick]
    o[np.arange(n), a] = A[pick, a]                              # exactly on the plane
    d = rng.normal(size=(n, 3))
    sgn = np.sign(nrm[pick, a])
    eps = rng.choice(np.array([0.0, 2.5e-8, 1e-7, 1e-6]), n)
    d[np.arange(n), a] = 0.0
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[np.arange(n), a] = sgn * eps
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3], rays[:, 4:7], rays[:, 7] = o, d, 1e35
    return rays, pick.astype(np.int32)
