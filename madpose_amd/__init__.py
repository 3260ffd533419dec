"""madpose_amd -- MI355X-native hybrid-RANSAC relative pose with monocular depth priors.

Drop-in for the Python API of kocurvik/madpose (`import madpose` resolves to this
package through the thin `madpose/` alias).  Minimal samples are solved and every
hypothesis is scored on the GPU (HIP kernels for gfx950); local optimisation runs on
the host.  See DESIGN.md.
"""
from .api import (  # noqa: F401
    EstimatorConfig,
    HybridEstimatePoseAndScale,
    HybridEstimatePoseScaleOffset,
    HybridEstimatePoseScaleOffsetSharedFocal,
    HybridEstimatePoseScaleOffsetTwoFocal,
    HybridLORansacOptions,
    HybridRansacStatistics,
    LORansacOptions,
    PoseAndScale,
    PoseScaleOffset,
    PoseScaleOffsetSharedFocal,
    PoseScaleOffsetTwoFocal,
    RansacOptions,
    RansacStats,
    device_count,
    estimate_batch,
    estimate_scale_and_pose,
    bougnoux_focals_batch,
    lm_refine_batch,
    get_depths_batch,
    pose_auc_batch,
    pose_eval_batch,
    profile_enable,
    profile_read,
    profile_reset,
    relpose_5pt,
    relpose_6pt_shared_focal,
    relpose_7pt_two_focal,
    score_models,
    set_device,
    solve_scale_and_shift,
    solve_scale_and_shift_shared_focal,
    solve_scale_and_shift_two_focal,
    solve_scale_shift_pose,
    solve_scale_shift_pose_shared_focal,
    solve_scale_shift_pose_ours,
    solve_scale_shift_pose_shared_focal_ours,
    solve_scale_shift_pose_two_focal,
    solve_scale_shift_pose_two_focal_4p4d,
    solve_scale_shift_pose_two_focal_ours,
    version,
)
from . import utils  # noqa: F401

__all__ = [n for n in dir() if not n.startswith("_")]
