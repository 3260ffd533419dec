"""Writes tests/golden/lm_gauge_cal.json: a calibrated EPI_ONLY LO problem (Sampson
residuals alone) on which the engine's host LM and the oracle end at the same cost but
at different |t| and a rotation 6e-6 deg apart -- the gauge drift behind the EPI_ONLY
tolerance of tests/lm_cases.py close() (1e-3 deg rotation, 1e-4 t direction;
tests/test_lm_host_cpu.py::test_lm_gauge_fixture).  The problem is the 61st draw of
tests/lm_cases.problems for (variant 0, non-monotonic steps, LO_type 1); this script
finds it by its index and stores its index lists, start model, both end models and
their costs."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import madpose  # noqa: E402
from tests import lm_cases as LC  # noqa: E402

INDEX = 60


def _d(m):
    return {"R": np.asarray(m["R"] if isinstance(m, dict) else m.R()).tolist(),
            "t": np.asarray(m["t"] if isinstance(m, dict) else m.t()).tolist(),
            "scale": float(m["scale"] if isinstance(m, dict) else m.scale),
            "offset0": float(m["offset0"] if isinstance(m, dict) else m.offset0),
            "offset1": float(m["offset1"] if isinstance(m, dict) else m.offset1), "focal0": 1.0, "focal1": 1.0}


def main():
    variant, nonmono, lo_type = 0, True, 1
    rng = np.random.default_rng(100 + variant)
    p, o, c, args, norm_scale, est = LC.setup(variant, nonmono, lo_type)
    cands = LC.problems(rng, p, variant, norm_scale, 96, est)
    kind, lists, m0 = cands[INDEX]
    (ref, ran, reason), = LC.classify(variant, args, o, c, [cands[INDEX]], lo_type)
    assert ran and reason is None
    (mh, st), = madpose.lm_refine_batch(variant, *args, o, c, [cands[INDEX]], on_host=True)
    out = {"variant": variant, "nonmono": nonmono, "lo_type": lo_type, "kind": int(kind), "index": INDEX,
           "lists": [[int(i) for i in l] for l in lists], "start": _d(m0), "oracle": _d(ref), "host": _d(mh),
           "start_cost": LC.lm_cost(variant, args, o, c, m0, lists, norm_scale),
           "oracle_cost": LC.lm_cost(variant, args, o, c, LC.model_of(ref, variant), lists, norm_scale),
           "host_cost": LC.lm_cost(variant, args, o, c, mh, lists, norm_scale)}
    with open(os.path.join(ROOT, "tests", "golden", "lm_gauge_cal.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
