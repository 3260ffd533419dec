"""Pre/post-processing helpers of the reference's Python package (madpose/utils.py).

Same names and semantics (pinned by tests/test_utils_cpu.py and tests/test_get_depths_gpu.py against outputs of the
reference recorded in tests/golden/utils.npz), plus the SuperGlue-style pose AUC used
for the ScanNet-1500-style evaluation (not in the reference).
"""
import numpy as np


def get_depths(image, depth_map, mkpts):
    """Nearest-neighbour depth lookup (madpose/utils.py:4-22): keypoints are rescaled
    from image to depth-map resolution, rounded half-to-even, clipped, then indexed [y, x]."""
    dm_h, dm_w = depth_map.shape[:2]
    im_h, im_w = image.shape[:2]
    factor = np.array([dm_w / im_w, dm_h / im_h])
    ij = np.round(np.asarray(mkpts) * factor).astype(int)
    cols = np.clip(ij[:, 0], 0, dm_w - 1)
    rows = np.clip(ij[:, 1], 0, dm_h - 1)
    return depth_map[rows, cols]


def bougnoux_numpy(F, p1, p2):
    """Bougnoux focal lengths from a fundamental matrix (madpose/utils.py:25-56).
    Returns the squared focals (f1^2, f2^2) as the reference does."""
    a = np.r_[np.asarray(p1, dtype=np.float64).reshape(2), 1.0][:, None]
    b = np.r_[np.asarray(p2, dtype=np.float64).reshape(2), 1.0][:, None]
    U, _, Vt = np.linalg.svd(F, full_matrices=True)
    e1 = Vt[2, :] / Vt[2, 2]
    e2 = U[:, 2] / U[2, 2]

    def cross_mat(v):
        return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])

    I2 = np.diag([1.0, 1.0, 0.0])
    S1, S2 = cross_mat(e1), cross_mat(e2)
    f1 = (-b.T @ S2 @ I2 @ F @ (a @ a.T) @ F.T @ b) / (b.T @ S2 @ I2 @ F @ I2 @ F.T @ b)
    f2 = (-a.T @ S1 @ I2 @ F.T @ (b @ b.T) @ F @ a) / (a.T @ S1 @ I2 @ F.T @ I2 @ F @ a)
    return f1[0, 0], f2[0, 0]


def angle_error_mat(R1, R2):
    """Rotation angle between R1 and R2 in degrees (madpose/utils.py:59-62)."""
    c = np.clip((np.trace(R1.T @ R2) - 1.0) / 2.0, -1.0, 1.0)
    return np.rad2deg(np.abs(np.arccos(c)))


def angle_error_vec(v1, v2):
    """Angle between two vectors in degrees (madpose/utils.py:65-67)."""
    n = np.linalg.norm(v1) * np.linalg.norm(v2)
    return np.rad2deg(np.arccos(np.clip(np.dot(v1, v2) / n, -1.0, 1.0)))


def compute_pose_error(T_0to1, R, t, t_thres=None):
    """(translation angle, rotation angle) in degrees (madpose/utils.py:70-78); the
    translation error is folded to [0, 90] because E only fixes t up to sign."""
    R_gt, t_gt = T_0to1[:3, :3], T_0to1[:3, 3]
    et = angle_error_vec(t, t_gt)
    et = np.minimum(et, 180.0 - et)
    eR = angle_error_mat(R, R_gt)
    if t_thres is not None and np.linalg.norm(t_gt) < t_thres:
        et = 0
    return et, eR


def pose_auc(errors, thresholds=(5, 10, 20)):
    """Area under the cumulative pose-error curve up to each threshold (degrees),
    with errors = max(err_R, err_t) per pair (SuperGlue evaluation convention)."""
    errors = np.sort(np.asarray(errors, dtype=np.float64))
    recall = (np.arange(len(errors)) + 1) / len(errors)
    errors = np.r_[0.0, errors]
    recall = np.r_[0.0, recall]
    aucs = []
    for t in thresholds:
        last = np.searchsorted(errors, t)
        r = np.r_[recall[:last], recall[last - 1]]
        e = np.r_[errors[:last], t]
        aucs.append(np.trapezoid(r, x=e) / t)
    return aucs
