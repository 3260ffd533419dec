"""Device get_depths (madpose/utils.py:4-22) for many pairs in one
launch, bit-identical to the reference's numpy code: the golden fixture captured from
the reference (tests/golden/utils.npz) and random maps, keypoints and size ratios,
including points outside the image (clipping) and near-.5 products (round half to
even)."""
import os

import numpy as np
import pytest

import madpose
from madpose_amd import utils

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module", autouse=True)
def require_gpu():
    if madpose.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")


def test_golden_fixture():
    g = np.load(os.path.join(GOLDEN, "utils.npz"))
    img = tuple(int(v) for v in g["gd_image_shape"][:2])
    (out,) = madpose.get_depths_batch([img], [g["gd_depthmap"]], [g["gd_kpts"]])
    assert out.dtype == g["gd_out"].dtype and np.array_equal(out, g["gd_out"])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_random_batch_matches_numpy(dtype):
    rng = np.random.default_rng(4)
    imgs, maps, kps = [], [], []
    for p in range(40):
        ih, iw = rng.integers(200, 1100, 2)
        dh, dw = rng.integers(50, 700, 2)
        n = int(rng.integers(0, 3000))
        kp = np.c_[rng.uniform(-20, iw + 20, n), rng.uniform(-20, ih + 20, n)]
        if n:  # keypoints that land exactly on .5 after scaling (ties to even)
            kp[: n // 10, 0] = (np.floor(kp[: n // 10, 0]) + 0.5) * iw / dw
        imgs.append((int(ih), int(iw)))
        maps.append(rng.uniform(0.1, 80.0, (int(dh), int(dw))).astype(dtype))
        kps.append(kp)
    outs = madpose.get_depths_batch(imgs, maps, kps)
    for img, dm, kp, out in zip(imgs, maps, kps, outs):
        ref = utils.get_depths(np.zeros(img), dm, kp)
        assert out.dtype == dm.dtype and np.array_equal(out, ref)

