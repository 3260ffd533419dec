"""Synthetic correspondence sets with known ground truth.

There is no dataset access offline; configs 2-5 of BASELINE.json are reproduced with
these generators (seeded numpy default_rng), shaped like the reference's benchmarks:
ScanNet-like intrinsics, depth priors that are an affine distortion of the true
depths with multiplicative noise, pixel noise and uniformly random outliers.
"""
import numpy as np

SCANNET_K = np.array([[577.87, 0.0, 319.5], [0.0, 577.87, 239.5], [0.0, 0.0, 1.0]])


def _axis_angle(axis, ang):
    axis = axis / np.linalg.norm(axis)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


def make_pair(seed, n=2000, K0=None, K1=None, size0=(640, 480), size1=(640, 480), noise_px=1.0,
              outlier_ratio=0.3, depth_noise=0.05, rot_deg=(5.0, 30.0), t_norm=(0.2, 1.0)):
    """One synthetic image pair with n correspondences.

    Returns dict(x0, x1 [n x 2 pixels], depth0, depth1, min_depth, K0, K1, pp0, pp1,
    R, t, T_0to1, inlier_mask, f0, f1)."""
    rng = np.random.default_rng(seed)
    K0 = SCANNET_K.copy() if K0 is None else np.asarray(K0, dtype=np.float64)
    K1 = K0.copy() if K1 is None else np.asarray(K1, dtype=np.float64)
    R = _axis_angle(rng.standard_normal(3), np.deg2rad(rng.uniform(*rot_deg)))
    tdir = rng.standard_normal(3)
    t = tdir / np.linalg.norm(tdir) * rng.uniform(*t_norm)
    K0i = np.linalg.inv(K0)
    pts0, X0s, X1s = [], [], []
    need = n
    while need > 0:
        m = 4 * need + 64
        uv = np.c_[rng.uniform(0, size0[0], m), rng.uniform(0, size0[1], m)]
        z = rng.uniform(1.0, 8.0, m)
        rays = (K0i @ np.c_[uv, np.ones(m)].T).T
        X0 = rays * z[:, None]
        X1 = X0 @ R.T + t
        ok = X1[:, 2] > 0.1
        p1 = (K1 @ X1[ok].T).T
        p1 = p1[:, :2] / p1[:, 2:3]
        inside = (p1[:, 0] >= 0) & (p1[:, 0] < size1[0]) & (p1[:, 1] >= 0) & (p1[:, 1] < size1[1])
        sel = np.flatnonzero(ok)[inside][:need]
        pts0.append(uv[sel])
        X0s.append(X0[sel])
        X1s.append(X1[sel])
        need -= len(sel)
    x0 = np.concatenate(pts0)[:n]
    X0 = np.concatenate(X0s)[:n]
    X1 = np.concatenate(X1s)[:n]
    p1 = (K1 @ X1.T).T
    x1 = p1[:, :2] / p1[:, 2:3]
    x0 = x0 + noise_px * rng.standard_normal(x0.shape)
    x1 = x1 + noise_px * rng.standard_normal(x1.shape)
    n_out = int(round(outlier_ratio * n))
    out_idx = rng.choice(n, n_out, replace=False)
    inlier = np.ones(n, dtype=bool)
    inlier[out_idx] = False
    x1[out_idx] = np.c_[rng.uniform(0, size1[0], n_out), rng.uniform(0, size1[1], n_out)]
    z0, z1 = X0[:, 2].copy(), X1[:, 2].copy()
    z1[out_idx] = rng.uniform(1.0, 8.0, n_out)  # a prior looked up at a wrong location
    while True:
        a0, a1 = rng.uniform(0.5, 2.0, 2)
        b0 = rng.uniform(-0.3, 0.3) * np.median(z0)
        b1 = rng.uniform(-0.3, 0.3) * np.median(z1)
        d0 = (z0 - b0) / a0 * np.exp(depth_noise * rng.standard_normal(n))
        d1 = (z1 - b1) / a1 * np.exp(depth_noise * rng.standard_normal(n))
        if np.all(d0 > 0) and np.all(d1 > 0):
            break
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return dict(x0=x0, x1=x1, depth0=d0, depth1=d1, min_depth=np.array([d0.min(), d1.min()]), K0=K0, K1=K1,
                pp0=K0[:2, 2].copy(), pp1=K1[:2, 2].copy(), R=R, t=t, T_0to1=T, inlier_mask=inlier,
                f0=K0[0, 0], f1=K1[0, 0])


def config_pair(config, seed=0):
    """Pairs of BASELINE.json configs 2-4 (calibrated / shared-focal N=2000; two-focal N=4000)."""
    if config in ("calibrated", 2):
        return make_pair(seed, n=2000)
    if config in ("shared_focal", 3):
        return make_pair(seed, n=2000)
    if config in ("two_focal", 4):
        K0 = np.array([[618.96, 0, 539.5], [0, 618.96, 269.5], [0, 0, 1.0]])
        K1 = np.array([[374.91, 0, 479.5], [0, 374.91, 269.5], [0, 0, 1.0]])
        return make_pair(seed, n=4000, K0=K0, K1=K1, size0=(1080, 540), size1=(960, 540), noise_px=0.5,
                         outlier_ratio=0.2)
    raise ValueError(config)


def scannet_size(seed, n_range=(1500, 2500)):
    """Correspondence count of the configs[4] pair of this seed (cheap: no pair is built)."""
    return int(np.random.default_rng([7, seed]).integers(n_range[0], n_range[1] + 1))


def scannet_pair(seed, n_range=(1500, 2500)):
    """configs[4] stand-in (ScanNet-1500): a shared-focal pair
    with ScanNet intrinsics (f = 577.87, pp = ((W-1)/2, (H-1)/2)) and N ~ U{1500..2500}
    correspondences; the pair of seed s is the same whatever rank or batch draws it."""
    return make_pair(seed, n=scannet_size(seed, n_range))


def example_options(kind="calibrated", iterations=1000, min_iterations=100):
    """Options of examples/{calibrated,shared_focal,two_focal}.py (reference)."""
    from .api import EstimatorConfig, HybridLORansacOptions

    o = HybridLORansacOptions()
    o.min_num_iterations = min_iterations
    o.max_num_iterations = iterations
    o.final_least_squares = True
    o.threshold_multiplier = 5.0
    o.num_lo_steps = 4
    if kind == "two_focal":
        o.squared_inlier_thresholds = [16.0 ** 2, 1.0 ** 2]
    else:
        o.squared_inlier_thresholds = [8.0 ** 2, 2.0 ** 2]
    o.data_type_weights = [1.0, 1.0]
    o.random_seed = 0
    c = EstimatorConfig()
    c.min_depth_constraint = True
    c.use_shift = True
    return o, c


def throughput_options(kind="calibrated", iterations=100000):
    """Configs 2-4: fixed iteration count (min = max = max_per_solver), example LO settings."""
    o, c = example_options(kind, iterations=iterations, min_iterations=iterations)
    o.max_num_iterations_per_solver = iterations
    return o, c
