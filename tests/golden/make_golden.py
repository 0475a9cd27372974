"""Generate the golden fixtures under tests/golden/ (run here, where
/root/reference and oracle/_ref exist).

* box_box_annotation.json -- known-answer case transcribed from the
  reference's unittests/unit/test_DARTCollide.cpp:554
  (BOX_BOX_FACE_FACE_COLLISION_ANNOTATION): inputs and expected contacts.
* lcp_fixtures.json -- (a) boxed-LCP problems transcribed from the reference's
  unittests/unit/test_LCPUtils.cpp:198 (LCP_FAILURE_2); (b) random frictional
  contact LCPs (A = J Minv J^T, b, lo/hi/findex as ContactConstraint builds
  them) with the solution x produced by the reference's OWN Dantzig solver
  (dart/external/odelcpsolver compiled into oracle/_ref/libodelcp.so).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
INF = float("inf")


def enc(x):
    if isinstance(x, float) and not np.isfinite(x):
        return "inf" if x > 0 else "-inf"
    return x


def random_contact_lcp(rng, ncontacts, ndof):
    J = rng.standard_normal((3 * ncontacts, ndof))
    L = rng.standard_normal((ndof, ndof))
    Minv = L @ L.T + 0.1 * np.eye(ndof)
    A = J @ Minv @ J.T
    b = rng.standard_normal(3 * ncontacts) * 0.1
    mu = 1.0
    lo, hi, fi = [], [], []
    for c in range(ncontacts):
        lo += [0.0, -mu, -mu]
        hi += [INF, mu, mu]
        fi += [-1, 3 * c, 3 * c]
    return A, b, np.array(lo), np.array(hi), np.array(fi, dtype=np.int32)


def main():
    # --- box-box known answer -------------------------------------------------
    box = {
        "source": "unittests/unit/test_DARTCollide.cpp:554 BOX_BOX_FACE_FACE_COLLISION_ANNOTATION",
        "size1": [1.0, 1.0, 1.0], "T1_translation": [0.0, 0.0, -0.5],
        "size2": [0.5, 0.5, 0.5], "T2_translation": [0.0, 0.5, 0.25],
        "expected": [
            {"point": [0.25, 0.5, 0.0], "type": "EDGE_EDGE"},
            {"point": [-0.25, 0.5, 0.0], "type": "EDGE_EDGE"},
            {"point": [0.25, 0.25, 0.0], "type": "FACE_VERTEX"},
            {"point": [-0.25, 0.25, 0.0], "type": "FACE_VERTEX"},
        ],
    }
    with open(os.path.join(HERE, "box_box_annotation.json"), "w") as f:
        json.dump(box, f, indent=1)

    # --- LCP fixtures -----------------------------------------------------------
    probs = []
    A = np.array([
        [0.348223, 0.12244, 0, 0.223228, 0.122446, 0],
        [0.12244, 0.63095, 0, 0.37244, 0.630938, 0],
        [0, 0, 0, 0, 0, 0],
        [0.223228, 0.37244, 0, 0.348222, 0.372434, 0],
        [0.122446, 0.630938, 0, 0.372434, 0.630926, 0],
        [0, 0, 0, 0, 0, 0]])
    b = np.array([-0.0124998, 0.0250006, 0, 0.0124996, 0.0249994, 0])
    lo = np.array([0, -1, -1, 0, -1, -1.0])
    hi = np.array([INF, 1, 1, INF, 1, 1])
    fi = np.array([-1, 0, 0, -1, 3, 3], dtype=np.int32)
    probs.append(("test_LCPUtils.cpp:198 LCP_FAILURE_2", A, b, lo, hi, fi))
    rng = np.random.default_rng(1234)
    for k in range(40):
        nc = int(rng.integers(1, 9))
        nd = int(rng.integers(6, 34))
        A, b, lo, hi, fi = random_contact_lcp(rng, nc, nd)
        probs.append((f"random contact LCP #{k} ({nc} contacts, {nd} dofs)", A, b, lo, hi, fi))
    out = []
    for name, A, b, lo, hi, fi in probs:
        r = O.ref_dantzig(A, b, lo, hi, fi, early=False)
        if r is None:
            raise SystemExit("oracle/_ref/libodelcp.so missing: build with `make -C oracle ref`")
        ok, x = r
        out.append({"name": name, "A": A.tolist(), "b": b.tolist(), "lo": [enc(v) for v in lo.tolist()],
                    "hi": [enc(v) for v in hi.tolist()], "findex": fi.tolist(), "ref_success": ok,
                    "ref_x": x.tolist()})
    with open(os.path.join(HERE, "lcp_fixtures.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "solver": "reference dSolveLCP (dart/external/odelcpsolver/lcp.cpp) via oracle/_ref",
                   "problems": out}, f)
    print("wrote", len(out), "LCP fixtures")


if __name__ == "__main__":
    main()
