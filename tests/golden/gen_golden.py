"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (where /root/reference exists):

    python tests/golden/gen_golden.py

What it produces (all plain data, loadable with allow_pickle=False):

* md_solvers.npz  -- inputs and outputs of the reference's numpy prototypes of the
  three monocular-depth (MD) minimal solvers:
    solver_py/scale_and_shift.py:6-117              solve_shift_and_scale
    solver_py/scale_and_shift_shared_focal.py:6-294 solve_shift_and_scale_shared_focal
    solver_py/scale_and_shift_two_focal.py:6-353    solve_shift_and_scale_two_focal
  These prototypes use the same elimination templates as src/solver.cpp:35-480.
  Instances follow the instance generators of the reference's own self-checks
  (solver_py/scale_and_shift.py:131-155 and the shared/two-focal analogues), seeded.
* md_pose.npz     -- the pose stage of the MD solvers: every solution in md_solvers.npz
  that passes the positivity filter of src/solver.cpp:503-504 (704-705, 1008-1009)
  turned into (R, t, scale, offset0, offset1, focals) with the reference's own
  find_transform (solver_py/scale_and_shift.py:120-129, _shared_focal.py:297,
  _two_focal.py:356) on the corrected 3D points (image points divided by the focal(s)
  first, as src/solver.cpp:711-714 does).
* utils.npz       -- outputs of madpose/utils.py (get_depths, compute_pose_error,
  bougnoux_numpy) on the example pairs shipped in examples/image_pairs/.
* example_pairs.npz -- the example matches / intrinsics / GT poses (data files of the
  reference) plus the depth priors looked up with the reference get_depths, so that
  tests on the GPU box never read /root/reference.

The reference is imported only here; nothing in tests/ or the product imports it.
`import madpose` inside solver_py is stubbed because it is used there only for
cross-checks against the compiled extension (which cannot be built offline).
"""
import importlib.util
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _rand_rot(rng):
    R = np.linalg.qr(rng.standard_normal((3, 3)))[0]
    return R * np.linalg.det(R)


def md_instance(rng, npts, f0, f1, noise_px):
    """Random MD instance: returns (x_homo 3xK, y_homo 3xK, d_x, d_y, gt dict)."""
    while True:
        x1 = np.c_[rng.standard_normal((npts, 2)), np.ones(npts)]
        d1_gt = 1.0 + 5.0 * rng.random(npts)
        X = x1 * d1_gt[:, None]
        R = _rand_rot(rng)
        t = rng.standard_normal(3)
        X2 = X @ R.T + t
        d2_gt = X2[:, 2]
        x2 = X2 / d2_gt[:, None]
        if np.all(d2_gt > 0.1):
            break
    x1[:, :2] *= f0
    x2[:, :2] *= f1
    if noise_px > 0:
        x2[:, :2] += noise_px * rng.standard_normal((npts, 2))
    a1, b1 = 0.2 + rng.random(), rng.standard_normal()
    a2, b2 = 0.2 + rng.random(), rng.standard_normal()
    d1 = (d1_gt - b1) / a1
    d2 = (d2_gt - b2) / a2
    gt = dict(R=R, t=t, b1=b1 / a1, a2=a2 / a1, b2=b2 / a1, f0=f0, f1=f1)
    return x1.T.copy(), x2.T.copy(), d1, d2, gt


def gen_md(ss, ssf, stf, n_clean=150, n_noisy=50):
    out = {}
    specs = [
        ("cal", 3, ss.solve_shift_and_scale, 4, lambda r: (1.0, 1.0)),
        ("sf", 4, ssf.solve_shift_and_scale_shared_focal, 5, lambda r: (f := 300.0 + 900.0 * r.random(), f)),
        ("tf", 4, stf.solve_shift_and_scale_two_focal, 6, lambda r: (300.0 + 900.0 * r.random(), 300.0 + 900.0 * r.random())),
    ]
    for name, k, fn, width, focals in specs:
        rng = np.random.default_rng({"cal": 11, "sf": 12, "tf": 13}[name])
        X, Y, DX, DY, SOL, NSOL, NOISE = [], [], [], [], [], [], []
        GT = []
        for i in range(n_clean + n_noisy):
            noisy = i >= n_clean
            f0, f1 = focals(rng)
            noise = (0.5 if name != "cal" else 0.5 / 500.0) if noisy else 0.0
            xh, yh, dx, dy, gt = md_instance(rng, k, f0, f1, noise)
            # reference prototype takes row-stacked points (K x 3)
            sols = fn(xh.T.copy(), yh.T.copy(), dx.copy(), dy.copy())
            sols = [np.real(np.asarray(s, dtype=np.complex128)).astype(np.float64) for s in sols]
            buf = np.full((8, width), np.nan)
            for j, s in enumerate(sols[:8]):
                buf[j, : len(s)] = s
            X.append(xh)
            Y.append(yh)
            DX.append(dx)
            DY.append(dy)
            SOL.append(buf)
            NSOL.append(len(sols))
            NOISE.append(noise)
            GT.append([gt["b1"], gt["a2"], gt["b2"], gt["f0"], gt["f1"]] + list(gt["R"].ravel()) + list(gt["t"]))
        out[f"{name}_x"] = np.array(X)
        out[f"{name}_y"] = np.array(Y)
        out[f"{name}_dx"] = np.array(DX)
        out[f"{name}_dy"] = np.array(DY)
        out[f"{name}_sols"] = np.array(SOL)
        out[f"{name}_nsols"] = np.array(NSOL, dtype=np.int32)
        out[f"{name}_noise"] = np.array(NOISE)
        out[f"{name}_gt"] = np.array(GT)
    np.savez_compressed(os.path.join(OUT, "md_solvers.npz"), **out)
    print("md_solvers.npz:", {k: v.shape for k, v in out.items() if k.endswith("_sols")})


def gen_md_pose(ss, ssf, stf):
    md = np.load(os.path.join(OUT, "md_solvers.npz"))
    out = {}
    for name, ft in (("cal", ss.find_transform), ("sf", ssf.find_transform), ("tf", stf.find_transform)):
        X, Y, DX, DY = md[f"{name}_x"], md[f"{name}_y"], md[f"{name}_dx"], md[f"{name}_dy"]
        SOL, NS = md[f"{name}_sols"], md[f"{name}_nsols"]
        poses = np.full((len(X), 8, 17), np.nan)
        count = np.zeros(len(X), dtype=np.int32)
        for i in range(len(X)):
            k = 0
            for j in range(min(int(NS[i]), 8)):
                s_ = SOL[i, j]
                b1, a2, b2 = s_[1], s_[2], s_[3]
                d1 = DX[i] + b1
                d2 = DY[i] * a2 + b2
                if d1.min() <= 0 or d2.min() <= 0:  # src/solver.cpp:503-504
                    continue
                f0 = f1 = 1.0
                if name == "sf":
                    f0 = f1 = s_[4]
                elif name == "tf":
                    f0, f1 = s_[4], s_[5]
                xu, yu = X[i].copy(), Y[i].copy()
                xu[:2] /= f0
                yu[:2] /= f1
                R, t = ft((xu * d1[None, :]).T, (yu * d2[None, :]).T)
                poses[i, k] = np.r_[R.ravel(), t, a2, b1, b2, f0, f1]
                k += 1
            count[i] = k
        out[f"{name}_pose"] = poses
        out[f"{name}_npose"] = count
    np.savez_compressed(os.path.join(OUT, "md_pose.npz"), **out)
    print("md_pose.npz:", {k: int(v.sum()) for k, v in out.items() if k.endswith("_npose")})


def gen_examples(utils):
    out = {}
    util_out = {}
    pairs = {
        "eth3d": ("1_eth3d", True),
        "2d3ds": ("2_2d3ds", True),
        "scannet": ("0_scannet", False),
    }
    for key, (folder, has_depth) in pairs.items():
        base = os.path.join(REF, "examples", "image_pairs", folder)
        with open(os.path.join(base, "info.json")) as f:
            info = json.load(f)
        m0 = np.load(os.path.join(base, info["matches_0_file"]))
        m1 = np.load(os.path.join(base, info["matches_1_file"]))
        out[f"{key}_m0"] = m0.astype(np.float64)
        out[f"{key}_m1"] = m1.astype(np.float64)
        out[f"{key}_K0"] = np.array(info["K0"], dtype=np.float64)
        out[f"{key}_K1"] = np.array(info["K1"], dtype=np.float64)
        out[f"{key}_T"] = np.array(info["T_0to1"], dtype=np.float64)
        if has_depth:
            dm0 = np.load(os.path.join(base, info["depth_0_file"]))
            dm1 = np.load(os.path.join(base, info["depth_1_file"]))
            # the images only provide their shape to get_depths; read it from the png header
            shp0 = _png_shape(os.path.join(base, "image0.png"))
            shp1 = _png_shape(os.path.join(base, "image1.png"))
            img0 = np.zeros(shp0 + (3,), dtype=np.uint8)
            img1 = np.zeros(shp1 + (3,), dtype=np.uint8)
            out[f"{key}_img0_shape"] = np.array(shp0)
            out[f"{key}_img1_shape"] = np.array(shp1)
            out[f"{key}_depth0"] = utils.get_depths(img0, dm0, m0).astype(np.float64)
            out[f"{key}_depth1"] = utils.get_depths(img1, dm1, m1).astype(np.float64)
            out[f"{key}_mindepth"] = np.array([dm0.min(), dm1.min()], dtype=np.float64)
            # small crops of the depth maps (for get_depths parity on the GPU box)
            util_out[f"{key}_dm0_shape"] = np.array(dm0.shape)
            util_out[f"{key}_dm0_crop"] = dm0[::8, ::8].astype(np.float64)
    # get_depths on synthetic inputs with a resize factor (exercises rounding / clipping)
    rng = np.random.default_rng(5)
    dm = rng.random((37, 53)).astype(np.float32)
    img = np.zeros((111, 160, 3), dtype=np.uint8)
    kp = np.c_[rng.uniform(-3, 163, 400), rng.uniform(-3, 114, 400)]
    kp[:5] = [[0, 0], [159.5, 110.5], [160.4, 111.6], [-0.6, 50.5], [80.5, -0.5]]
    util_out["gd_depthmap"] = dm
    util_out["gd_image_shape"] = np.array(img.shape)
    util_out["gd_kpts"] = kp
    util_out["gd_out"] = utils.get_depths(img, dm, kp)
    # pose errors
    errs = []
    Rs, ts, Ts = [], [], []
    for i in range(50):
        T = np.eye(4)
        T[:3, :3] = _rand_rot(rng)
        T[:3, 3] = rng.standard_normal(3)
        R = _rand_rot(rng) if i % 3 == 0 else T[:3, :3] @ _small_rot(rng, 0.05 * i)
        t = T[:3, 3] + 0.1 * rng.standard_normal(3) * (i % 5)
        if i % 7 == 0:
            t = -t
        et, eR = utils.compute_pose_error(T, R, t)
        errs.append([et, eR])
        Rs.append(R)
        ts.append(t)
        Ts.append(T)
    util_out["pe_T"] = np.array(Ts)
    util_out["pe_R"] = np.array(Rs)
    util_out["pe_t"] = np.array(ts)
    util_out["pe_err"] = np.array(errs)
    # bougnoux
    Fs, pp, fo = [], [], []
    for i in range(30):
        K0 = np.diag([400 + 400 * rng.random(), 0, 1.0])
        K0[1, 1] = K0[0, 0]
        K1 = np.diag([400 + 400 * rng.random(), 0, 1.0])
        K1[1, 1] = K1[0, 0]
        R = _rand_rot(rng)
        t = rng.standard_normal(3)
        E = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]]) @ R
        F = np.linalg.inv(K1).T @ E @ np.linalg.inv(K0)
        p1 = rng.standard_normal(2) * 5
        p2 = rng.standard_normal(2) * 5
        Fs.append(F)
        pp.append(np.r_[p1, p2])
        fo.append(utils.bougnoux_numpy(F, p1, p2))
    util_out["bg_F"] = np.array(Fs)
    util_out["bg_pp"] = np.array(pp)
    util_out["bg_out"] = np.array(fo)
    np.savez_compressed(os.path.join(OUT, "example_pairs.npz"), **out)
    np.savez_compressed(os.path.join(OUT, "utils.npz"), **util_out)
    print("example_pairs.npz:", sorted(out))


def _small_rot(rng, ang):
    a = rng.standard_normal(3)
    a = a / np.linalg.norm(a) * ang
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    th = np.linalg.norm(a)
    if th == 0:
        return np.eye(3)
    K = K / th
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def _png_shape(path):
    with open(path, "rb") as f:
        head = f.read(24)
    w = int.from_bytes(head[16:20], "big")
    h = int.from_bytes(head[20:24], "big")
    return (h, w)


def main():
    sys.modules.setdefault("madpose", types.ModuleType("madpose"))
    ss = _load(os.path.join(REF, "solver_py", "scale_and_shift.py"), "ref_ss")
    ssf = _load(os.path.join(REF, "solver_py", "scale_and_shift_shared_focal.py"), "ref_ssf")
    stf = _load(os.path.join(REF, "solver_py", "scale_and_shift_two_focal.py"), "ref_stf")
    utils = _load(os.path.join(REF, "madpose", "utils.py"), "ref_utils")
    if "--pose-only" not in sys.argv:
        gen_md(ss, ssf, stf)
        gen_examples(utils)
    gen_md_pose(ss, ssf, stf)


if __name__ == "__main__":
    main()
