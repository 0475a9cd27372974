"""LCPUtils (dart/constraint/LCPUtils.cpp) in the oracle, pinned by the
reference's own test cases (unittests/unit/test_LCPUtils.cpp, transcribed in
tests/golden/lcp_utils_cases.json by make_lcp_utils_golden.py) and, where the
reference's Dantzig solver is built (oracle/_ref), by running it.  CPU only."""
import json
import os

import numpy as np
import pytest

import models
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _dec(v):
    return np.array([float("inf") if x == "inf" else float("-inf") if x == "-inf" else x for x in v])


def _cases():
    return {c["name"].split()[-1]: c for c in json.load(open(os.path.join(GOLD, "lcp_utils_cases.json")))["cases"]}


def _prob(c):
    return (np.array(c["A"]), np.array(c["x"], float), np.array(c["b"], float), _dec(c["lo"]), _dec(c["hi"]),
            np.array(c["findex"], np.int32))


def _lower_sym(A):
    return np.tril(A) + np.tril(A, -1).T


def test_reduce_real_life_failure_1(oracle_built):
    """REAL_LIFE_FAILURE_1 (:423): reduce == merges (0,3), (1,3), (2,3)."""
    c = _cases()["REAL_LIFE_FAILURE_1"]
    A, x, b, lo, hi, fi = _prob(c)
    # the reference calls reduce(A, x, lo, hi, b, fIndex): lo in b's place
    Ar, xr, br, hr, lr, fr, mp = O.lcp_reduce(A, x, lo, hi, b, fi)
    assert np.allclose(Ar, np.array(c["expect"]["reduced_A"]), atol=1e-8)
    assert fr.tolist() == c["expect"]["reduced_findex"] and mp.tolist() == c["expect"]["map"]
    # with the arguments in signature order the merge pattern is the same
    Ar2, *_rest, mp2 = O.lcp_reduce(A, x, b, hi, lo, fi)
    assert np.array_equal(Ar2, Ar) and np.array_equal(mp2, mp)


def test_merge_cols_then_dantzig(oracle_built):
    """MERGE_COLS (:51): merging (0,2) then (1,2) and solving the 2x2 with
    Dantzig (early termination) succeeds, and mapOut x is valid for the
    original problem."""
    c = _cases()["MERGE_COLS"]
    A, x, b, lo, hi, fi = _prob(c)
    Ar, xr, br, hr, lr, fr, mp = O.lcp_reduce(A, x, b, hi, lo, fi)
    assert mp.tolist() == [0, 1, 0, 1]  # reduce finds exactly the test's merges
    ok, xs = O.dantzig(_lower_sym(Ar), br, lr, hr, fr, True)
    assert ok
    assert O.lcp_valid(A, xs[mp], b, hi, lo, fi)
    ref = O.ref_dantzig(Ar, br, lr, hr, fr, True)
    if ref is not None:  # the reference's own solver on the non-symmetric reduced A
        assert ref[0] and np.allclose(ref[1], xs, rtol=1e-12, atol=1e-15)


def test_solve_merged(oracle_built):
    """SOLVE_MERGED (:124): LCPUtils::solveDeduplicated (reduce, Dantzig
    without early termination, validity, mapOut) succeeds and is valid."""
    c = _cases()["SOLVE_MERGED"]
    A, x, b, lo, hi, fi = _prob(c)
    x0 = O.cod_solve(A, b)
    Ar, xr, br, hr, lr, fr, mp = O.lcp_reduce(A, x0, b, hi, lo, fi)
    assert len(br) < len(b)
    ok, xs = O.dantzig(_lower_sym(Ar), br, lr, hr, fr, False)
    assert ok
    assert O.lcp_valid(A, xs[mp], b, hi, lo, fi)


def test_lcp_failure_pgs(oracle_built):
    """LCP_FAILURE (:370): guessSolution then PGS with Option(50000, 1e-15,
    1e-12, 1e-10) gives a valid solution."""
    c = _cases()["LCP_FAILURE"]
    A, x, b, lo, hi, fi = _prob(c)
    g = O.guess_solution(A, b, fi)
    ok, xs = O.pgs(A, g, b, lo, hi, fi, options=c["expect"]["pgs_option"])
    assert O.lcp_valid(A, xs, b, hi, lo, fi)


def test_lcp_failure_2_remove_friction(oracle_built):
    """LCP_FAILURE_2 (:198): removeFriction then PGS, valid with friction
    ignored."""
    c = _cases()["LCP_FAILURE_2"]
    A, x, b, lo, hi, fi = _prob(c)
    keep = np.where(fi == -1)[0]
    Ar = A[np.ix_(keep, keep)]
    ok, xs = O.pgs(Ar, x[keep], b[keep], lo[keep], hi[keep], np.full(len(keep), -1), options=c["expect"]["pgs_option"])
    assert O.lcp_valid(Ar, xs, b[keep], hi[keep], lo[keep], np.full(len(keep), -1), True)


def test_dantzig_reads_lower_triangle(oracle_built):
    """ODE's dLCP reads only the lower triangle of the row-major A it is given
    (lcp.cpp:144 swapRowsAndCols, matrix.cpp:371 GETA) -- the property the
    reduced (column-doubled, non-symmetric) problems rely on.  Checked on the
    reference's compiled solver: REAL_LIFE_FAILURE_2 (:467, a non-symmetric
    matrix from the reference) and reduced contact LCPs with duplicated
    contacts; the restatement, given the mirrored lower triangle, matches."""
    if O.ref_lib() is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    c = _cases()["REAL_LIFE_FAILURE_2"]
    A, x, b, lo, hi, fi = _prob(c)
    probs = [(A, b, lo, hi, fi)]
    rng = np.random.default_rng(1)
    for _ in range(150):
        # contact LCPs with duplicated contacts (repeated J rows, as coincident
        # contact points give), reduced by LCPUtils::reduce: the non-symmetric
        # problems the fallback solve actually hands to dLCP
        nc, nd = int(rng.integers(2, 8)), int(rng.integers(4, 20))
        J = rng.standard_normal((3 * nc, nd))
        for k in range(int(rng.integers(1, nc))):
            src, dst = rng.choice(nc, 2, replace=False)
            J[3 * dst:3 * dst + 3] = J[3 * src:3 * src + 3]
        L = rng.standard_normal((nd, nd))
        A = J @ (L @ L.T + 0.05 * np.eye(nd)) @ J.T
        bb = (J @ rng.standard_normal(nd)) * 0.2
        lo, hi = np.tile([0.0, -1.0, -1.0], nc), np.tile([np.inf, 1.0, 1.0], nc)
        fi = np.array([v for k in range(nc) for v in (-1, 3 * k, 3 * k)], np.int32)
        Ar, _x, br, hr, lr, fr, _mp = O.lcp_reduce(A, np.zeros(3 * nc), bb, hi, lo, fi)
        assert len(br) < 3 * nc
        probs.append((Ar, br, lr, hr, fr))
    for A, b, lo, hi, fi in probs:
        for early in (False, True):
            r1 = O.ref_dantzig(A, b, lo, hi, fi, early)
            r2 = O.ref_dantzig(_lower_sym(A), b, lo, hi, fi, early)
            o = O.dantzig(_lower_sym(A), b, lo, hi, fi, early)
            assert r1[0] == r2[0] == o[0]
            if r1[0]:
                assert np.array_equal(r1[1], r2[1])
                assert np.allclose(o[1], r1[1], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("name", ["MERGE_COLS", "SOLVE_MERGED", "LCP_FAILURE", "LCP_FAILURE_2",
                                  "REAL_LIFE_FAILURE_1", "REAL_LIFE_FAILURE_4", "REAL_LIFE_FAILURE_5",
                                  "BLOCK_SYMMETRIC_CASE"])
def test_cascade_on_reference_cases(oracle_built, name):
    """BoxedLcpConstraintSolver::solveLcp's fallback cascade on the reference's
    cases: the result satisfies the LCP it claims to solve (Dantzig: A; PGS:
    A + cfm I; frictionless: the normal rows), and duplicate columns are
    merged wherever the case has them."""
    c = _cases()[name]
    A, x, b, lo, hi, fi = _prob(c)
    xs, path, reduced, ign, cfm = O.lcp_cascade(A, b, lo, hi, fi, x)
    assert np.isfinite(xs).all()
    dup = len(O.lcp_reduce(A, x, b, hi, lo, fi)[2]) < len(b)
    assert reduced == dup
    if path == 0:
        assert O.lcp_valid(A, xs, b, hi, lo, fi)
    elif path == 1:
        assert O.lcp_valid(A + cfm * np.eye(len(b)), xs, b, hi, lo, fi)
    else:
        assert ign and (xs[fi >= 0] == 0).all()


def test_classify_probe_matches_the_oracle_step():
    """oracle.classify (the short-circuit classification + standardisation on
    a raw problem, Q from A's entries), which the GPU parity tests perturb to
    probe whether a world's short-circuit split is ambiguous, reproduces the
    oracle step's own short-circuit outcome on every contact world of an
    Atlas and a resting-box batch (no warm start: guessSolution)."""
    for mk, states in ((lambda: models.atlas_world(True),
                        lambda w: models.random_states(w, 96, seed=3, q_scale=0.01, v_scale=0.02)),
                       (models.box_world, lambda w: models.box_states("rest", 32, seed=5))):
        w = mk()
        st, f = states(w)
        ow = O.OracleWorld(w)
        ow.forward(st, f)
        seen = 0
        for b in range(st.shape[0]):
            A, bb, lo, hi, fi = O.lcp_problem(ow, b)
            if len(bb) == 0:
                continue
            ok, _ = O.classify(A, bb, lo, hi, fi, O.guess_solution(A, bb, fi))
            assert ok == bool(O.lcp_flags(ow, b)[0]), b
            seen += 1
        assert seen > 20
