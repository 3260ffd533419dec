"""Three-way LM comparison on the LM parity test problems: the engine host LM (no device
needed) against the oracle; diagnostic."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, oracle, madpose, sys
from madpose_amd import synthetic
from tests.helpers import oracle_cfg, oracle_opts, rot_angle_deg
from tests.test_lm_device_gpu import _problems, _oracle_model, KIND
def run(variant, nonmono, lo_type):
    rng = np.random.default_rng(100 + variant)
    p = synthetic.make_pair(40 + variant, n=800) if variant < 2 else synthetic.config_pair(4, seed=40)
    o, c = synthetic.example_options(KIND[variant], iterations=100)
    c.ceres_use_nonmonotonic_steps = nonmono
    c.LO_type = lo_type
    cam0, cam1 = (p["K0"], p["K1"]) if variant == 0 else (p["pp0"], p["pp1"])
    args = (p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], cam0, cam1)
    _, _, ns = oracle.score_models(variant, *args[:4], cam0, cam1, oracle_opts(o), oracle_cfg(c), [])
    m, st, _ = oracle.estimate(variant, *args, oracle_opts(o), oracle_cfg(synthetic.example_options(KIND[variant], iterations=100)[1]))
    mk = [madpose.PoseScaleOffset, madpose.PoseScaleOffsetSharedFocal, madpose.PoseScaleOffsetTwoFocal][variant]
    extra = [[], [m['focal0']], [m['focal0'], m['focal1']]][variant]
    est = mk(m['R'], m['t'], m['scale'], m['offset0'], m['offset1'], *extra)
    probs = _problems(rng, p, variant, ns, 24, est)
    on_dev = "--device" in sys.argv
    got = madpose.lm_refine_batch(variant, *args, o, c, probs, on_host=True)
    dev = madpose.lm_refine_batch(variant, *args, o, c, probs) if on_dev else got
    bad = []
    for j, ((kind, lists, m0), (mm, st), (md, sd)) in enumerate(zip(probs, got, dev)):
        ref, ran = oracle.least_squares(variant, *args, oracle_opts(o), oracle_cfg(c), kind, lists, _oracle_model(m0, variant))
        if not ran: continue
        eh = rot_angle_deg(mm.R(), ref['R'])
        ed = rot_angle_deg(md.R(), ref['R'])
        ehd = rot_angle_deg(md.R(), mm.R())
        oh = abs(mm.offset0 - ref['offset0']) / (1 + abs(ref['offset0']))
        od = abs(md.offset0 - ref['offset0']) / (1 + abs(ref['offset0']))
        if max(eh, ed) > 1e-6 or max(oh, od) > 1e-7:
            bad.append((j, kind, [len(l) for l in lists], "host-oracle %.1e/%.1e dev-oracle %.1e/%.1e dev-host %.1e"
                        % (eh, oh, ed, od, ehd), round(ref['offset0'], 4)))
    print(variant, nonmono, lo_type, 'bad:', bad, flush=True)
for v in (0, 1, 2):
    for nm, lt in [(True, 0), (False, 0), (True, 1), (True, 2)]:
        run(v, nm, lt)
