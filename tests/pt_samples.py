"""Minimal samples of the point solvers for the root-stage parity tests
(tests/test_pt_roots_gpu.py, tests/test_oracle_cpu.py): normalized image points
(identity intrinsics), K points per sample, in four kinds:

  random     noise-free and noisy random scenes (points in front of both cameras);
  outlier    correspondences drawn across the image in both views independently
             (a sample of a contaminated match set), and inlier samples with one to
             three of their points replaced by such draws;
  wide       coordinates, depths and baselines spanning decades (wide fields of view,
             near and far points, tiny and large translations);
  neardouble samples on which the oracle's real-root count changes: a sample is moved
             along a straight path towards another one and the path parameter where
             the count changes is bisected to 2^-44 -- there two real roots merge (or
             one escapes to infinity), the ill-conditioned case of any root finder.

Bearings are formed as the estimator forms them from (u, v, 1) with identity
intrinsics: b = x / sqrt((u u + v v) + 1), the same IEEE operations as the device."""
import numpy as np


def _rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def bearings(p):
    """(..., K, 2) normalized points -> (..., K, 3) unit bearings, the estimator's operations."""
    u, v = p[..., 0], p[..., 1]
    n = np.sqrt((u * u + v * v) + 1.0)
    return np.stack([u / n, v / n, 1.0 / n], axis=-1)


def _small_rot(rng, max_angle):
    w = rng.normal(size=3)
    w *= rng.uniform(0, max_angle) / np.linalg.norm(w)
    th = np.linalg.norm(w)
    k = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]]) / th
    return np.eye(3) + np.sin(th) * k + (1 - np.cos(th)) * (k @ k)


def _scene(rng, K, spread=1.0, depth=(2.0, 6.0), tscale=1.0, noise=0.0, max_angle=None):
    for _ in range(1000):
        R = _rot(rng) if max_angle is None else _small_rot(rng, max_angle)
        t = rng.normal(size=3)
        t *= tscale / np.linalg.norm(t)
        X = np.c_[rng.uniform(-spread, spread, (K, 2)), rng.uniform(*depth, K)]
        X[:, :2] *= X[:, 2:]
        Y = X @ R.T + t
        if np.all(Y[:, 2] > 1e-3):
            p0 = X[:, :2] / X[:, 2:]
            p1 = Y[:, :2] / Y[:, 2:]
            if noise:
                p0 = p0 + rng.normal(scale=noise, size=p0.shape)
                p1 = p1 + rng.normal(scale=noise, size=p1.shape)
            return p0, p1
    raise RuntimeError("no scene in front of both cameras")


def random_samples(rng, ns, K):
    out0, out1 = np.zeros((ns, K, 2)), np.zeros((ns, K, 2))
    for s in range(ns):
        out0[s], out1[s] = _scene(rng, K, noise=0.0 if s % 2 == 0 else 0.01)
    return out0, out1


def outlier_samples(rng, ns, K):
    out0, out1 = np.zeros((ns, K, 2)), np.zeros((ns, K, 2))
    for s in range(ns):
        if s % 2 == 0:  # every point an outlier: uniform across a 90-degree field of view
            out0[s] = rng.uniform(-1, 1, (K, 2))
            out1[s] = rng.uniform(-1, 1, (K, 2))
        else:
            p0, p1 = _scene(rng, K, noise=0.002)
            k = rng.integers(1, 4)
            idx = rng.choice(K, size=k, replace=False)
            p1[idx] = rng.uniform(-1, 1, (k, 2))
            out0[s], out1[s] = p0, p1
    return out0, out1


def wide_samples(rng, ns, K):
    out0, out1 = np.zeros((ns, K, 2)), np.zeros((ns, K, 2))
    for s in range(ns):
        m = s % 4
        if m == 0:  # very wide field of view
            out0[s], out1[s] = _scene(rng, K, spread=10.0 ** rng.uniform(0, 1.5), max_angle=0.3)
        elif m == 1:  # depths over four decades
            out0[s], out1[s] = _scene(rng, K, depth=(0.05, 500.0), max_angle=0.5)
        elif m == 2:  # tiny or huge baseline
            out0[s], out1[s] = _scene(rng, K, tscale=10.0 ** rng.uniform(-5, 2))
        else:  # narrow field of view, far scene
            out0[s], out1[s] = _scene(rng, K, spread=10.0 ** rng.uniform(-3, -1), depth=(10.0, 1000.0),
                                      tscale=10.0 ** rng.uniform(-2, 1))
    return out0, out1


def near_double_samples(rng, ns, K, count, tries=60):
    """count(p0, p1) -> number of real roots (the oracle's); bisection of the path
    parameter between two samples with different counts, to 2^-44."""
    out0, out1 = [], []
    while len(out0) < ns:
        a0, a1 = _scene(rng, K, noise=0.01) if rng.random() < 0.5 else (rng.uniform(-1, 1, (K, 2)),
                                                                          rng.uniform(-1, 1, (K, 2)))
        b0, b1 = _scene(rng, K, noise=0.01)
        ca, cb = count(a0, a1), count(b0, b1)
        if ca == cb:
            continue
        lo, hi = 0.0, 1.0
        for _ in range(44):
            mid = 0.5 * (lo + hi)
            cm = count((1 - mid) * a0 + mid * b0, (1 - mid) * a1 + mid * b1)
            if cm == ca:
                lo = mid
            else:
                hi = mid
        for lam in (lo, hi):
            out0.append((1 - lam) * a0 + lam * b0)
            out1.append((1 - lam) * a1 + lam * b1)
    return np.array(out0[:ns]), np.array(out1[:ns])


def all_kinds(seed, ns, K, count):
    rng = np.random.default_rng(seed)
    return {"random": random_samples(rng, ns, K), "outlier": outlier_samples(rng, ns, K),
            "wide": wide_samples(rng, ns, K), "neardouble": near_double_samples(rng, ns, K, count)}
