"""configs[4] (ScanNet-1500 stand-in) through the batched path: many pairs in flight
on one device (mp_estimate_batch) must give every pair the oracle's result, so the
per-pair pose errors and the pose AUC@5/10/20 equal the CPU oracle's (BASELINE.json:
"pose AUC@5 parity").  Smaller pairs than the bench (N ~ U{300..500}) keep the oracle
fast; the pose-error and AUC code is pinned by tests/test_utils_cpu.py."""
import numpy as np
import pytest

import madpose
import oracle
from madpose_amd import synthetic, utils
from tests.helpers import oracle_cfg, oracle_opts, rot_angle_deg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def require_gpu():
    if madpose.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")


def test_batch_pose_auc_matches_oracle():
    pairs = [synthetic.scannet_pair(s, n_range=(300, 500)) for s in range(16)]
    o, c = synthetic.example_options("shared_focal", iterations=300)
    res = madpose.estimate_batch(1, pairs, o, c, num_streams=6)
    e_dev, e_orc = [], []
    for p, (m, st) in zip(pairs, res):
        ref, rst, inl = oracle.estimate(1, p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], p["pp0"],
                                        p["pp1"], oracle_opts(o), oracle_cfg(c))
        assert st.num_iterations_total == rst.num_iterations_total
        assert st.num_hypotheses == rst.num_hypotheses, (st.num_hypotheses, rst.num_hypotheses)
        assert rot_angle_deg(m.R(), ref["R"]) <= 1e-6
        for t in range(3):
            assert np.array_equal(np.sort(st.inlier_indices[t]), np.sort(inl[t]))
        e_dev.append(max(utils.compute_pose_error(p["T_0to1"], m.R(), m.t())))
        e_orc.append(max(utils.compute_pose_error(p["T_0to1"], ref["R"], ref["t"])))
    assert np.allclose(e_dev, e_orc, rtol=0, atol=1e-6)
    auc_dev = utils.pose_auc(e_dev, (5, 10, 20))
    auc_orc = utils.pose_auc(e_orc, (5, 10, 20))
    assert np.allclose(auc_dev, auc_orc, rtol=0, atol=1e-6), (auc_dev, auc_orc)
    assert auc_dev[2] > 0.5  # the synthetic set is solvable


def _oracle_scannet(seed):
    """One stand-in pair through the CPU oracle (a worker of the process pool below: a
    fresh interpreter that never touches the GPU)."""
    p = synthetic.scannet_pair(seed)
    o, c = synthetic.example_options("shared_focal", iterations=1000)
    ref, rst, inl = oracle.estimate(1, p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], p["pp0"],
                                    p["pp1"], oracle_opts(o), oracle_cfg(c))
    return (rst.num_iterations_total, rst.number_lo_iterations, np.asarray(ref["R"]), np.asarray(ref["t"]),
            [np.sort(np.asarray(x)) for x in inl])


def test_full_size_scannet_pairs_match_oracle():
    """configs[4] at its own sizes: all 1500 pairs of the stand-in set (seeds 0..1499,
    N ~ U{1500..2500}, the bench's example options with 1000 iterations) with 8 pairs in
    flight, as bench.py runs them; every pair equals the oracle's (the oracle runs in a
    pool of spawned CPU processes), and the device pose evaluator (mp_pose_eval) gives
    the oracle poses' AUC@5/10/20 over the whole set."""
    import multiprocessing
    import os
    from concurrent.futures import ProcessPoolExecutor

    n_pairs = 1500
    workers = max(1, min(12, (os.cpu_count() or 2) - 1))
    with ProcessPoolExecutor(max_workers=workers, mp_context=multiprocessing.get_context("spawn")) as ex:
        refs = list(ex.map(_oracle_scannet, range(n_pairs), chunksize=25))
    pairs = [synthetic.scannet_pair(s) for s in range(n_pairs)]
    o, c = synthetic.example_options("shared_focal", iterations=1000)
    res = madpose.estimate_batch(1, pairs, o, c, num_streams=8)
    Ro, to = [], []
    for k, (p, (m, st)) in enumerate(zip(pairs, res)):
        its, nlo, R_ref, t_ref, inl = refs[k]
        assert st.num_iterations_total == its, k
        assert st.number_lo_iterations == nlo, k
        assert rot_angle_deg(m.R(), R_ref) <= 1e-6, k
        for t in range(3):
            assert np.array_equal(np.sort(st.inlier_indices[t]), inl[t]), k
        Ro.append(R_ref)
        to.append(t_ref)
    T = np.stack([p["T_0to1"] for p in pairs])
    R = np.stack([np.asarray(m.R()) for m, _ in res])
    t = np.stack([np.asarray(m.t()).reshape(3) for m, _ in res])
    _, _, auc_dev = madpose.pose_eval_batch(T, R, t, (5, 10, 20))
    e_orc = [max(utils.compute_pose_error(T[k], Ro[k], to[k])) for k in range(len(pairs))]
    assert np.allclose(auc_dev, utils.pose_auc(e_orc, (5, 10, 20)), rtol=0, atol=1e-6)
