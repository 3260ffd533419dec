"""CPU tests of the oracle itself: pinned against the reference's golden vectors."""
import os

import numpy as np
import pytest

import oracle
from madpose_amd import synthetic
from tests.helpers import oracle_cfg, oracle_opts, rot_angle_deg, solution_sets_match

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("variant,name", [(0, "cal"), (1, "sf"), (2, "tf")])
def test_oracle_md_matches_reference_goldens(variant, name):
    g = np.load(os.path.join(GOLDEN, "md_solvers.npz"))
    for i in range(len(g[f"{name}_x"])):
        ref = g[f"{name}_sols"][i, : g[f"{name}_nsols"][i]]
        ref = ref[np.all(np.isfinite(ref), axis=1)]
        mine = oracle.md_scale_shift(variant, g[f"{name}_x"][i].T, g[f"{name}_y"][i].T, g[f"{name}_dx"][i],
                                     g[f"{name}_dy"][i])
        ok, err = solution_sets_match(ref, mine, 1e-6)
        assert ok, (name, i, err)


@pytest.mark.parametrize("variant,name", [(0, "cal"), (1, "sf"), (2, "tf")])
def test_oracle_md_recovers_ground_truth(variant, name):
    """Noise-free golden instances: one root equals the generating (b1, a2, b2, f)."""
    g = np.load(os.path.join(GOLDEN, "md_solvers.npz"))
    noise = g[f"{name}_noise"]
    for i in np.flatnonzero(noise == 0)[:60]:
        gt = g[f"{name}_gt"][i]
        sols = oracle.md_scale_shift(variant, g[f"{name}_x"][i].T, g[f"{name}_y"][i].T, g[f"{name}_dx"][i],
                                     g[f"{name}_dy"][i])
        want = [gt[0], gt[1], gt[2]] + ([gt[3]] if variant == 1 else [gt[3], gt[4]] if variant == 2 else [])
        errs = [np.max(np.abs(s[1:] - want) / (1 + np.abs(want))) for s in sols]
        assert min(errs) < 1e-6, (i, errs)


def test_oracle_5pt_recovers_ground_truth():
    rng = np.random.default_rng(0)
    for _ in range(40):
        R = np.linalg.qr(rng.standard_normal((3, 3)))[0]
        R *= np.linalg.det(R)
        t = rng.standard_normal(3)
        X = np.c_[rng.uniform(-1, 1, (5, 2)), rng.uniform(2, 6, 5)]
        X2 = X @ R.T + t
        if np.any(X2[:, 2] < 0.1):
            continue
        b1 = X / np.linalg.norm(X, axis=1, keepdims=True)
        b2 = X2 / np.linalg.norm(X2, axis=1, keepdims=True)
        poses = oracle.relpose_5pt(b1, b2)
        tn = t / np.linalg.norm(t)
        err = min(rot_angle_deg(p["R"], R) + np.abs(p["t"] / np.linalg.norm(p["t"]) - tn).max() for p in poses)
        assert err < 1e-5  # degrees + unit-vector difference


def test_oracle_estimator_recovers_pose():
    p = synthetic.make_pair(0, n=400)
    o, c = synthetic.example_options("calibrated", iterations=300)
    m, st, inl = oracle.estimate(0, p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], p["K0"], p["K1"],
                                 oracle_opts(o), oracle_cfg(c))
    assert rot_angle_deg(m["R"], p["R"]) < 0.5
    assert st.number_lo_iterations >= 1
    # inlier lists are sorted, unique and within range
    for t in range(3):
        assert np.all(np.diff(inl[t]) > 0) and (len(inl[t]) == 0 or inl[t][-1] < 400)
    # true inliers dominate the returned set
    frac = np.mean(p["inlier_mask"][inl[2]])
    assert frac > 0.9


def test_oracle_alt_solvers_recover_ground_truth():
    """use_ours / use_4p4d restatements (oracle/src/md_alt.cpp) on noise-free instances."""
    rng = np.random.default_rng(0)
    hits = {"cal": 0, "sf": 0, "tf": 0}
    n = 60
    for _ in range(n):
        while True:
            R = np.linalg.qr(rng.standard_normal((3, 3)))[0]
            R *= np.linalg.det(R)
            t = rng.standard_normal(3) * 0.5
            X = np.c_[rng.uniform(-1, 1, (4, 2)), rng.uniform(2, 6, 4)]
            Y = X @ R.T + t
            if np.all(Y[:, 2] > 0.5):
                break
        u, v, s = rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5), rng.uniform(0.5, 2)
        sols = oracle.md_pose_alt(0, 1, (X / X[:, 2:])[:3], (Y / Y[:, 2:])[:3], X[:3, 2] - u, Y[:3, 2] / s - v)
        hits["cal"] += any(np.abs(m["R"] - R).max() < 1e-6 and abs(m["offset0"] - u) < 1e-6 for m in sols)
        f0, f1 = rng.uniform(0.5, 3, 2)
        xs = np.c_[f0 * X[:, :2] / X[:, 2:], np.ones(4)]
        sols = oracle.md_pose_alt(1, 1, xs, np.c_[f0 * Y[:, :2] / Y[:, 2:], np.ones(4)], X[:, 2], Y[:, 2] / s)
        hits["sf"] += any(np.abs(m["R"] - R).max() < 1e-6 and abs(m["focal0"] - f0) < 1e-6 for m in sols)
        sols = oracle.md_pose_alt(2, 1, xs, np.c_[f1 * Y[:, :2] / Y[:, 2:], np.ones(4)], X[:, 2], Y[:, 2] / s)
        hits["tf"] += any(abs(m["focal0"] - f0) < 1e-6 and abs(m["focal1"] - f1) < 1e-6 for m in sols)
    # the calibrated solver drops roots that the reference's column bookkeeping loses
    assert hits["cal"] >= 0.9 * n and hits["sf"] == n and hits["tf"] == n, hits


@pytest.mark.parametrize("variant,name", [(0, "cal"), (1, "sf"), (2, "tf")])
def test_oracle_md_pose_matches_reference_find_transform(variant, name):
    """The oracle's MD pose stage against md_pose.npz (reference find_transform on the
    reference prototypes' roots, positivity filter of src/solver.cpp:503-504)."""
    g = np.load(os.path.join(GOLDEN, "md_solvers.npz"))
    gp = np.load(os.path.join(GOLDEN, "md_pose.npz"))
    checked = 0
    for i in range(len(g[f"{name}_x"])):
        x, y, dx, dy = g[f"{name}_x"][i], g[f"{name}_y"][i], g[f"{name}_dx"][i], g[f"{name}_dy"][i]
        mine = oracle.md_pose(variant, x.T, y.T, dx, dy)
        k = int(gp[f"{name}_npose"][i])
        ref = gp[f"{name}_pose"][i, :k]
        # noisy instances: the reference's LAPACK roots themselves carry ~1e-7 relative
        # error on the worst-conditioned two-focal systems, which the pose inherits
        tol = 1e-4 if g[f"{name}_noise"][i] > 0 else 1e-6
        assert len(mine) == k, (i, len(mine), k)
        for p in mine:
            r = ref[int(np.argmin(np.abs(ref[:, 13] - p["offset0"])))]
            assert rot_angle_deg(p["R"], r[:9].reshape(3, 3)) < tol, i
            np.testing.assert_allclose(p["t"], r[9:12], rtol=tol, atol=1e-8)
            assert abs(p["scale"] - r[12]) <= tol * (1 + abs(r[12]))
            assert abs(p["offset1"] - r[14]) <= tol * (1 + abs(r[14]))
            checked += 1
    assert checked > 200


# ---- round 6: the point solvers' restatements (oracle/src/pt_poselib.cpp) ----
import sys  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pt_samples as ps  # noqa: E402


def test_oracle_5pt_poselib_restatement_agrees_with_action_matrix_form():
    """The estimator's 5pt restatement (Nister + PoseLib's Sturm bisection) against the
    independent action-matrix form kept from round 2, on benign samples: equal pose
    counts, and 97 % of the poses within 1e-6 (PoseLib's Newton stage is unguarded and
    stops at |f| < 1e-10 on the monic polynomial: the roots of a close pair come out less
    accurate, and now and then Newton leaves the isolating interval for the pair's other
    root -- PoseLib's behaviour, restated)."""
    rng = np.random.default_rng(17)
    p0, p1 = ps.random_samples(rng, 600, 5)
    p0, p1 = p0[::2], p1[::2]  # the noise-free half
    b0, b1 = ps.bearings(p0), ps.bearings(p1)
    close = 0
    for s in range(len(b0)):
        new = oracle.relpose_5pt(b0[s], b1[s])
        old = oracle.relpose_5pt_action(b0[s], b1[s])
        assert len(new) == len(old), s
        for m in new:
            d = min(np.abs(m["R"] - o["R"]).max() + np.abs(m["t"] - o["t"]).max() for o in old)
            close += d < 1e-6
    assert close >= 0.97 * sum(len(oracle.relpose_5pt(b0[s], b1[s])) for s in range(len(b0)))


def test_oracle_5pt_root_stage_counts_on_hard_samples():
    """The real-root count of det B(z) is even for a degree-10 polynomial with simple
    roots; the E list has one matrix per root unless (x, y) is not finite -- on the hard
    kinds the restatement returns no more than ten and keeps its roots ascending."""
    kinds = ps.all_kinds(5, 150, 5, lambda a, b: len(oracle.relpose_5pt_E(ps.bearings(a), ps.bearings(b))[1]))
    for kind, (p0, p1) in kinds.items():
        for s in range(len(p0)):
            E, roots = oracle.relpose_5pt_E(ps.bearings(p0[s]), ps.bearings(p1[s]))
            assert len(E) <= len(roots) <= 10, (kind, s)
            assert np.all(np.diff(roots) > 0), (kind, s, roots)


def test_oracle_7pt_restatement_agrees_with_svd_form():
    rng = np.random.default_rng(19)
    p0, p1 = ps.random_samples(rng, 400, 7)
    b0, b1 = ps.bearings(p0), ps.bearings(p1)
    for s in range(len(b0)):
        F, G = oracle.relpose_7pt(b0[s], b1[s]), oracle.relpose_7pt_svd(b0[s], b1[s])
        assert len(F) == len(G), s
        for f in F:
            assert min(min(np.abs(f - g).max(), np.abs(f + g).max()) for g in G) < 1e-6, s


@pytest.mark.parametrize("roots", [(1.0, 2.0, 3.0), (-5.0, 0.25, 40.0), (0.5, 0.5 + 1e-3, -2.0)])
def test_oracle_solve_cubic_real_three_roots(roots):
    r1, r2, r3 = roots
    c2, c1, c0 = -(r1 + r2 + r3), r1 * r2 + r1 * r3 + r2 * r3, -r1 * r2 * r3
    got = np.sort(oracle.solve_cubic_real(c2, c1, c0))
    assert len(got) == 3
    assert np.allclose(got, np.sort(roots), atol=1e-6)


def test_oracle_solve_cubic_real_one_root():
    # (x - 2)(x^2 + 1)
    got = oracle.solve_cubic_real(-2.0, 1.0, -2.0)
    assert len(got) == 1 and abs(got[0] - 2.0) < 1e-12


@pytest.mark.parametrize("rank", [3, 2, 1])
def test_oracle_eigen_svd3_is_an_svd(rank):
    """the Eigen JacobiSVD restatement (la.cpp eigen_jacobi_svd3, which the
    device's mdx::svd3 follows bit for bit) checked on its own -- U and V orthogonal,
    U diag(s) V^T reconstructs A with s = diag(U^T A V) >= 0 descending -- on full-rank,
    rank-2 and rank-1 inputs.  Parity with Eigen itself stays unpinned (not vendored)."""
    rng = np.random.default_rng(rank)
    for _ in range(200):
        A = sum(np.outer(rng.normal(size=3), rng.normal(size=3)) * 10.0 ** rng.uniform(-3, 3) for _ in range(rank))
        U, V = oracle.eigen_svd3(A)
        assert np.abs(U.T @ U - np.eye(3)).max() < 1e-12
        assert np.abs(V.T @ V - np.eye(3)).max() < 1e-12
        S = U.T @ A @ V
        s = np.diag(S)
        scale = np.abs(A).max()
        assert np.abs(S - np.diag(s)).max() <= 1e-12 * scale
        assert np.all(s >= -1e-12 * scale) and np.all(np.diff(s) <= 1e-12 * scale)
        assert np.abs(U @ np.diag(s) @ V.T - A).max() <= 1e-12 * scale
        if rank < 3:
            assert abs(s[2]) <= 1e-12 * scale
