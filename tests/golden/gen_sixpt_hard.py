"""Builds tests/golden/sixpt_hard.json: the shared-focal 6pt samples on which the
device root stage and the oracle once disagreed (the JSON lines the diagnostic
tools/diag_pt67.py recorded under profiles/r02 and profiles/r03), each with the
positive real roots u of q(u) = det(u^2 M0 + u M1 + M2) / u^5 computed in 60-digit
arithmetic (mpmath) from a double-precision pencil of the sample.

The pencil here is a plain numpy restatement of the 6pt construction (the 3 x 3
null space of the epipolar constraints, the determinant and trace constraints as
polynomials in the null-space coordinates; PoseLib relpose_6pt_shared_focal, the
solver /root/reference/src/hybrid_pose_shared_focal_estimator.cpp:87 calls).  Roots
that lie closer than 1e-6 (relative) to another root or to the real axis's complex
neighbours are marked ill-posed: their count is not determined by double-precision
input, and the tests do not pin it.

Run: python tests/golden/gen_sixpt_hard.py   (needs mpmath; writes the JSON)."""
import glob
import json
import os
import sys

import mpmath as mp
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
K_MONO = [(3, 0), (2, 1), (1, 2), (0, 3), (2, 0), (1, 1), (0, 2), (1, 0), (0, 1), (0, 0)]


def bearings(p):
    p = np.asarray(p, float)
    return np.hstack([p, np.ones((len(p), 1))])


def _mul(a, b):
    r = {}
    for (i, j), u in a.items():
        for (p, q), v in b.items():
            if i + j + p + q <= 3:
                r[(i + p, j + q)] = r.get((i + p, j + q), 0.0) + u * v
    return r


def _add(a, b, s=1.0):
    r = dict(a)
    for k, v in b.items():
        r[k] = r.get(k, 0.0) + s * v
    return r


def pencil(b1, b2):
    """M[a] (10 x 10): rows = det F and the 9 entries of 2 F F^T W F - tr(F F^T W) F with
    W = diag(1, 1, w), coefficients of w^a; columns = the cubic monomials of (x, y)."""
    A = np.array([[b2[i][r] * b1[i][c] for r in range(3) for c in range(3)] for i in range(6)])
    _, _, vt = np.linalg.svd(np.vstack([A, np.zeros((3, 9))]))
    V = vt.T
    F = [{(1, 0): V[e, 6], (0, 1): V[e, 7], (0, 0): V[e, 8]} for e in range(9)]

    def f(r, c):
        return F[3 * r + c]

    det = {}
    det = _add(det, _mul(f(0, 0), _add(_mul(f(1, 1), f(2, 2)), _mul(f(1, 2), f(2, 1)), -1)))
    det = _add(det, _mul(f(0, 1), _add(_mul(f(1, 0), f(2, 2)), _mul(f(1, 2), f(2, 0)), -1)), -1)
    det = _add(det, _mul(f(0, 2), _add(_mul(f(1, 0), f(2, 1)), _mul(f(1, 1), f(2, 0)), -1)))
    Ga = [[_add(_mul(f(r, 0), f(s, 0)), _mul(f(r, 1), f(s, 1))) for s in range(3)] for r in range(3)]
    Gb = [[_mul(f(r, 2), f(s, 2)) for s in range(3)] for r in range(3)]
    tr0 = _add(Ga[0][0], Ga[1][1])
    tr1 = _add(_add(Gb[0][0], Gb[1][1]), Ga[2][2])
    tr2 = Gb[2][2]
    M = np.zeros((3, 10, 10))
    for k, ij in enumerate(K_MONO):
        M[0, 0, k] = det.get(ij, 0.0)
    for r in range(3):
        for c in range(3):
            T0 = _add(_mul(Ga[r][0], f(0, c)), _mul(Ga[r][1], f(1, c)))
            T0 = _add(_add(T0, T0), _mul(tr0, f(r, c)), -1)
            T1 = _add(_add(_mul(Gb[r][0], f(0, c)), _mul(Gb[r][1], f(1, c))), _mul(Ga[r][2], f(2, c)))
            T1 = _add(_add(T1, T1), _mul(tr1, f(r, c)), -1)
            T2 = _mul(Gb[r][2], f(2, c))
            T2 = _add(_add(T2, T2), _mul(tr2, f(r, c)), -1)
            for k, ij in enumerate(K_MONO):
                M[0, 1 + 3 * r + c, k] = T0.get(ij, 0.0)
                M[1, 1 + 3 * r + c, k] = T1.get(ij, 0.0)
                M[2, 1 + 3 * r + c, k] = T2.get(ij, 0.0)
    return M


def exact_roots(M, dps=60):
    """All roots of q (60 digits): the 16 coefficients by an exact-arithmetic DFT of the
    determinant on the unit circle, then mpmath polyroots."""
    mp.mp.dps = dps
    Ms = [mp.matrix(M[a].tolist()) for a in range(3)]
    qv = []
    for j in range(16):
        u = mp.expjpi(mp.mpf(2 * j) / 16)
        qv.append(mp.det(Ms[0] * u * u + Ms[1] * u + Ms[2]) / u ** 5)
    c = [sum((qv[j] * mp.expjpi(-mp.mpf(2 * j * k) / 16)).real for j in range(16)) / 16 for k in range(16)]
    while c and abs(c[-1]) < mp.mpf(10) ** (-dps + 5):
        c.pop()
    return mp.polyroots(c[::-1], maxsteps=2000, extraprec=1000)


def main():
    recs, seen = [], set()
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r0*", "**", "diag_pt67*.jsonl"), recursive=True))
    files += sorted(glob.glob(os.path.join(ROOT, "profiles", "r0*", "**", "diag*.log"), recursive=True))
    for fn in files:
        for line in open(fn):
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            if d.get("solver") != "6pt" or "p0" not in d:
                continue
            key = json.dumps([d["p0"], d["p1"]])
            if key in seen:
                continue
            seen.add(key)
            M = pencil(bearings(d["p0"]), bearings(d["p1"]))
            rts = exact_roots(M)
            pos = sorted(float(mp.re(r)) for r in rts
                         if abs(mp.im(r)) <= mp.mpf(10) ** -25 * max(1, abs(r)) and mp.re(r) > 0)
            # ill-posed: a positive real root within 1e-6 (relative) of another root
            ill = False
            for r in rts:
                if abs(mp.im(r)) <= mp.mpf(10) ** -25 * max(1, abs(r)) and mp.re(r) > 0:
                    near = [s for s in rts if s is not r and abs(s - r) <= 1e-6 * abs(r)]
                    ill = ill or bool(near)
            recs.append({"origin": os.path.relpath(fn, ROOT) + f" trial {d.get('trial')} seed {d.get('seed')}",
                         "p0": d["p0"], "p1": d["p1"], "f_gt": d.get("f_gt"), "roots_u": pos, "ill_posed": ill})
            print(recs[-1]["origin"], len(pos), "roots", "ill-posed" if ill else "", flush=True)
    with open(os.path.join(HERE, "sixpt_hard.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_sixpt_hard.py", "samples": recs}, f, indent=1)
    print(len(recs), "samples")


if __name__ == "__main__":
    sys.exit(main())
