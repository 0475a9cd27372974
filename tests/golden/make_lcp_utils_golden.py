"""Generate tests/golden/lcp_utils_cases.json: the boxed-LCP cases of the
reference's unittests/unit/test_LCPUtils.cpp as data (inputs + what the
reference asserts about them), for tests/test_lcp_utils.py.

Transcribed literally: LCP_FAILURE (:370), LCP_FAILURE_2 (:198),
REAL_LIFE_FAILURE_1 (:423), REAL_LIFE_FAILURE_2 (:467), REAL_LIFE_FAILURE_4
(:557), REAL_LIFE_FAILURE_5 (:656), BLOCK_SYMMETRIC_CASE (:698).

MERGE_COLS (:51) and SOLVE_MERGED (:124) draw their inputs with
Eigen::VectorXs::Random, i.e. x + (y - x) * rand() / RAND_MAX on [-1, 1]
per coefficient in index order with glibc's rand() -- unseeded (seed 1) for
MERGE_COLS, the test's first, and srand(42) for SOLVE_MERGED; the same
draws are reproduced here through libc.  (If the reference's Eigen drew
differently the inputs are still cases of the same construction, on which the
reference asserts success and validity.)

Expected outputs are what the reference test asserts: REAL_LIFE_FAILURE_1's
reduced A equals three sequential mergeLCPColumns (0,3), (1,3), (2,3) -- each
doubles one column of A[:3,:3] -- and MERGE_COLS / SOLVE_MERGED / LCP_FAILURE /
LCP_FAILURE_2 assert solver success and isLCPSolutionValid.  The cases
without assertions in the reference are parity inputs (oracle vs GPU).
"""
import ctypes
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
INF = float("inf")


def enc(v):
    return [("inf" if x > 0 else "-inf") if isinstance(x, float) and not np.isfinite(x) else x for x in v]


_libc = ctypes.CDLL("libc.so.6")
RAND_MAX = 2147483647


def eigen_random(n):
    return np.array([-1.0 + 2.0 * float(_libc.rand()) / RAND_MAX for _ in range(n)])


def merge_cols_case():
    # test_LCPUtils.cpp:51 MERGE_COLS (first test: glibc's initial seed)
    _libc.srand(1)
    blk = eigen_random(2)
    aFac = np.concatenate([blk, blk])
    A = np.outer(aFac, aFac)
    x = eigen_random(4)
    b = eigen_random(4)
    b[2:4] = b[0:2]
    hi = np.full(4, 1000.0); lo = np.zeros(4); fi = [-1, 0, -1, 2]
    hi[1] = hi[3] = 1.0; lo[1] = lo[3] = -1.0
    return {"name": "test_LCPUtils.cpp:51 MERGE_COLS", "A": A.tolist(), "x": x.tolist(), "b": b.tolist(),
            "lo": enc(lo.tolist()), "hi": enc(hi.tolist()), "findex": fi,
            "merges": [[0, 2], [1, 2]], "expect": {"dantzig_success": True, "valid": True}}


def solve_merged_case():
    # test_LCPUtils.cpp:124 SOLVE_MERGED
    _libc.srand(42)
    blk = eigen_random(2)
    aFac = np.concatenate([blk, blk])
    A = np.outer(aFac, aFac)
    x = eigen_random(4)
    x[2:4] = x[0:2]
    b = A @ x
    x = eigen_random(4)
    hi = np.full(4, 1000.0); lo = np.zeros(4); fi = [-1, 0, -1, 2]
    hi[1] = hi[3] = 1.0; lo[1] = lo[3] = -1.0
    return {"name": "test_LCPUtils.cpp:124 SOLVE_MERGED", "A": A.tolist(), "x": x.tolist(), "b": b.tolist(),
            "lo": enc(lo.tolist()), "hi": enc(hi.tolist()), "findex": fi,
            "expect": {"solve_deduplicated_success": True, "valid": True}}


def six(rows):
    return [list(map(float, r)) for r in rows]


CASES = [
    {"name": "test_LCPUtils.cpp:370 LCP_FAILURE",
     "A": six([[2.5, 0, -0.00500001, 1.5, 0, -0.00499901], [0, 2.9901, 0, 0, 1.9901, 0],
               [-0.00500001, 0, 2.4901, 0.00500099, 0, 2.4901], [1.5, 0, 0.00500099, 2.5, 0, 0.00499999],
               [0, 1.9901, 0, 0, 2.9901, 0], [-0.00499901, 0, 2.4901, 0.00499999, 0, 2.4901]]),
     "x": [0.0] * 6, "lo": [0, -10000, -10000, 0, -10000, -10000.0],
     "hi": [INF, 10000, 10000, INF, 10000, 10000.0], "b": [0.01, 0, -1e-08, 0.01, 0, -1e-08],
     "findex": [-1, 0, 0, -1, 3, 3],
     "expect": {"guess_then_pgs_valid": True, "pgs_option": [50000, 1e-15, 1e-12, 1e-10]}},
    {"name": "test_LCPUtils.cpp:198 LCP_FAILURE_2",
     "A": six([[0.348223, 0.12244, 0, 0.223228, 0.122446, 0], [0.12244, 0.63095, 0, 0.37244, 0.630938, 0],
               [0] * 6, [0.223228, 0.37244, 0, 0.348222, 0.372434, 0],
               [0.122446, 0.630938, 0, 0.372434, 0.630926, 0], [0] * 6]),
     "x": [0, 0, 0, 0.00965809, 0.00965809, 0], "lo": [0, -1, -1, 0, -1, -1.0], "hi": [INF, 1, 1, INF, 1, 1.0],
     "b": [-0.0124998, 0.0250006, 0, 0.0124996, 0.0249994, 0], "findex": [-1, 0, 0, -1, 3, 3],
     "expect": {"remove_friction_pgs_valid": True, "pgs_option": [50000, 1e-15, 1e-12, 1e-10]}},
    {"name": "test_LCPUtils.cpp:423 REAL_LIFE_FAILURE_1",
     "A": six([[0.0424296, -0.0139791, 0, 0.0424296, -0.0139791, 0], [-0.0139791, 0.0698999, 0, -0.0139791, 0.0698999, 0],
               [0] * 6, [0.0424296, -0.0139791, 0, 0.0424296, -0.0139791, 0],
               [-0.0139791, 0.0698999, 0, -0.0139791, 0.0698999, 0], [0] * 6]),
     "x": [0.0] * 6, "lo": [0, -1, -1, 0, -1, -1.0], "hi": [INF, 1, 1, INF, 1, 1.0],
     "b": [1.67162, 2.08376, 0, 1.67162, 2.08376, 0], "findex": [-1, 0, 0, -1, 3, 3],
     # the reference test calls reduce(A, x, lo, hi, b, fIndex) (b and lo
     # swapped against the signature) and asserts the result equals the
     # merges (0,3), (1,3), (2,3): A[:3,:3] with each column doubled
     "reduce_args": "swap_b_lo",
     "expect": {"reduced_A": six([[0.0848592, -0.0279582, 0], [-0.0279582, 0.1397998, 0], [0, 0, 0]]),
                "reduced_findex": [-1, 0, 0], "map": [0, 1, 2, 0, 1, 2]}},
    {"name": "test_LCPUtils.cpp:467 REAL_LIFE_FAILURE_2",
     "A": six([[1, -0.0279582, 0], [-0.329466, 0.1398, 0], [0, 0, 0]]),
     "x": [19.6988, 0, 0], "lo": [0, -1, -1.0], "hi": [INF, 1, 1.0], "b": [19.6988, 2.08376, 0],
     "findex": [-1, 0, 0], "expect": {"nonsymmetric": True}},
    {"name": "test_LCPUtils.cpp:557 REAL_LIFE_FAILURE_4",
     "A": six([[0.0923023, 0.0247589, 0, 0.0923023, 0.0247589, 0], [0.0247589, 0.0137374, 0, 0.0247589, 0.0137374, 0],
               [0] * 6, [0.0923023, 0.0247589, 0, 0.0923023, 0.0247589, 0],
               [0.0247589, 0.0137374, 0, 0.0247589, 0.0137374, 0], [0] * 6]),
     "x": [0.0270786, -0.0270786, 0, 0.0270786, -0.0270786, 0], "lo": [0, -1, -1, 0, -1, -1.0],
     "hi": [INF, 1, 1, INF, 1, 1.0], "b": [0.00365796, 0.000140769, 0, 0.00365796, 0.000140769, 0],
     "findex": [-1, 0, 0, -1, 3, 3], "merges": [[0, 3], [1, 3], [2, 3]], "expect": {}},
    {"name": "test_LCPUtils.cpp:656 REAL_LIFE_FAILURE_5",
     "A": six([
         [1.0591, -0.0531116, 0, 1.0591, -0.0531116, 0, 1.06715, -0.0532007, 0, 1.06715, -0.0532007, 0],
         [-0.0531116, 1.05186, 0, -0.0531116, 1.05186, 0, -0.0548259, 1.05188, 0, -0.0548259, 1.05188, 0],
         [0] * 12,
         [1.0591, -0.0531116, 0, 1.0591, -0.0531116, 0, 1.06715, -0.0532007, 0, 1.06715, -0.0532007, 0],
         [-0.0531116, 1.05186, 0, -0.0531116, 1.05186, 0, -0.0548259, 1.05188, 0, -0.0548259, 1.05188, 0],
         [0] * 12,
         [1.06715, -0.0548259, 0, 1.06715, -0.0548259, 0, 1.08506, -0.0550241, 0, 1.08506, -0.0550241, 0],
         [-0.0532007, 1.05188, 0, -0.0532007, 1.05188, 0, -0.0550241, 1.0519, 0, -0.0550241, 1.0519, 0],
         [0] * 12,
         [1.06715, -0.0548259, 0, 1.06715, -0.0548259, 0, 1.08506, -0.0550241, 0, 1.08506, -0.0550241, 0],
         [-0.0532007, 1.05188, 0, -0.0532007, 1.05188, 0, -0.0550241, 1.0519, 0, -0.0550241, 1.0519, 0],
         [0] * 12]),
     "x": [0.00426985, 7.49341e-05, 0, 0.00426985, 7.49341e-05, 0, 0, 0, 0, 0, 0, 0],
     "lo": [0, -1, -1] * 4, "hi": [INF, 1, 1] * 4,
     "b": [0.0090364, -0.000295916, 0, 0.0090364, -0.000295916, 0, -0.0139171, -4.19424e-05, 0, -0.0139171,
           -4.19424e-05, 0],
     "findex": [-1, 0, 0, -1, 3, 3, -1, 6, 6, -1, 9, 9], "expect": {}},
    {"name": "test_LCPUtils.cpp:698 BLOCK_SYMMETRIC_CASE",
     "A": six([[0.0923029, 0.0247581, 0, 0.0923029, 0.0247581, 0], [0.0247581, 0.0137368, 0, 0.0247581, 0.0137368, 0],
               [0] * 6, [0.0923029, 0.0247581, 0, 0.0923029, 0.0247581, 0],
               [0.0247581, 0.0137368, 0, 0.0247581, 0.0137368, 0], [0] * 6]),
     "x": [0.0491903, 0.00921924, 0, 0, 0, 0], "lo": [0, -1, -1, 0, -1, -1.0], "hi": [INF, 1, 1, INF, 1, 1.0],
     "b": [0.00365797, 0.000140734, 0, 0.00365797, 0.000140734, 0], "findex": [-1, 0, 0, -1, 3, 3], "expect": {}},
]


def main():
    cases = [merge_cols_case(), solve_merged_case()]
    for c in CASES:
        c = dict(c)
        c["lo"], c["hi"] = enc([float(v) for v in c["lo"]]), enc([float(v) for v in c["hi"]])
        cases.append(c)
    out = {"generator": "tests/golden/make_lcp_utils_golden.py",
           "source": "unittests/unit/test_LCPUtils.cpp (reference)", "cases": cases}
    with open(os.path.join(HERE, "lcp_utils_cases.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
