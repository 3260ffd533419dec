"""Writes tests/golden/lm_ridge_tf.json: the two-focal EPI_ONLY LO problem on which the
host LM left the oracle in round 3 (blocks [128, 52, 77]; see
tests/test_lm_host_cpu.py::test_lm_ridge_fixture).  The problem is the 30-somethingth
draw of tests/lm_cases.problems for that configuration; this script finds it by its
sizes and stores its index lists, start model and the oracle's costs."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from tests import lm_cases as LC  # noqa: E402
from tests.helpers import oracle_cfg, oracle_opts  # noqa: E402


def main():
    variant, nonmono, lo_type = 2, True, 1
    rng = np.random.default_rng(100 + variant)
    p, o, c, args, norm_scale, est = LC.setup(variant, nonmono, lo_type)
    for kind, lists, m0 in LC.problems(rng, p, variant, norm_scale, 96, est):
        if [len(x) for x in lists] != [128, 52, 77]:
            continue
        ref, _ = oracle.least_squares(variant, *args, oracle_opts(o), oracle_cfg(c), kind, lists,
                                      LC.oracle_model(m0, variant))
        out = {"variant": variant, "nonmono": nonmono, "lo_type": lo_type, "kind": int(kind),
               "lists": [[int(i) for i in l] for l in lists],
               "start": {"R": m0.R().tolist(), "t": m0.t().tolist(), "scale": m0.scale, "offset0": m0.offset0,
                         "offset1": m0.offset1, "focal0": m0.focal0, "focal1": m0.focal1},
               "start_cost": LC.lm_cost(variant, args, o, c, m0, lists, norm_scale),
               "oracle_cost": LC.lm_cost(variant, args, o, c, LC.model_of(ref, variant), lists, norm_scale)}
        with open(os.path.join(ROOT, "tests", "golden", "lm_ridge_tf.json"), "w") as f:
            json.dump(out, f, indent=1)
        return
    raise SystemExit("problem not found")


if __name__ == "__main__":
    main()
