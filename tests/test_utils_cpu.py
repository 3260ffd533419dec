"""madpose.utils parity against outputs of the reference's madpose/utils.py."""
import os

import numpy as np

from madpose_amd import utils

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_get_depths():
    g = np.load(os.path.join(GOLDEN, "utils.npz"))
    img = np.zeros(tuple(g["gd_image_shape"]), dtype=np.uint8)
    out = utils.get_depths(img, g["gd_depthmap"], g["gd_kpts"])
    assert np.array_equal(out, g["gd_out"])


def test_example_depth_priors():
    ex = np.load(os.path.join(GOLDEN, "example_pairs.npz"))
    assert ex["eth3d_m0"].shape == (193, 2) and ex["2d3ds_m0"].shape == (782, 2)
    assert np.all(ex["eth3d_depth0"] > 0)


def test_compute_pose_error():
    g = np.load(os.path.join(GOLDEN, "utils.npz"))
    for T, R, t, e in zip(g["pe_T"], g["pe_R"], g["pe_t"], g["pe_err"]):
        et, eR = utils.compute_pose_error(T, R, t)
        assert abs(et - e[0]) < 1e-9 and abs(eR - e[1]) < 1e-9


def test_bougnoux():
    g = np.load(os.path.join(GOLDEN, "utils.npz"))
    for F, pp, ref in zip(g["bg_F"], g["bg_pp"], g["bg_out"]):
        f1, f2 = utils.bougnoux_numpy(F, pp[:2], pp[2:])
        assert np.allclose([f1, f2], ref, rtol=1e-9)


def test_pose_auc():
    errs = np.array([0.0, 1.0, 2.0, 30.0])
    auc = utils.pose_auc(errs, [5, 10, 20])
    assert 0 < auc[0] < auc[1] < auc[2] <= 1
