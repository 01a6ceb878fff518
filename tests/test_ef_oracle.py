"""The canonical-order EarlyFusion oracle (oracle/ef_oracle.cpp) pinned on the CPU.

ef_oracle restates EarlyFusion's three per-feature scores (earlyfusion_traile.py:165-173) in the
one float32 order the HIP kernels follow, so the Da-TACOS-size GPU flow can be compared with it
by ==. Here it is pinned against the reference itself:
  * its CSMs against the golden vectors made by importing the reference's get_csm,
    get_csm_cosine and get_csm_blocked_oti (tests/golden/make_golden.py) at float32 tolerance
    (the reference's BLAS order differs), and bit for bit on integer-exact blocks, where every
    order gives the same float;
  * its OTI against the golden get_oti indices; its binarisation against the golden
    csm_to_binary outputs (tie case included);
  * its three scores against np_oracle's composition of the golden-pinned numpy restatements
    on integer-exact block features: equal;
  * the early score's chain (getWCSM x 3, sum, exp, binarise, SW): getWCSM against the golden
    getWCSM output, and bit for bit against an independent numpy statement of the canonical order
    (ascending k-smallest sums, correctly rounded exp); the early score against that composition
    on every pair and against the reference's own composition wherever its early matrix is
    separated at the kappa-NN boundary.
"""
import numpy as np
import pytest

import oracle
from oracle import np_oracle as npo
from conftest import GOLDEN


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("tag", ["s", "m"])
def test_ef_csm_golden(gold, tag):
    X, Y = gold["csm_%s_X" % tag], gold["csm_%s_Y" % tag]
    np.testing.assert_allclose(oracle.ef_csm(X, Y, 0), gold["csm_%s_euclid" % tag], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(oracle.ef_csm(X, Y, 1), gold["csm_%s_cosine" % tag], rtol=1e-5, atol=1e-5)


def test_ef_blocked_oti_golden(gold):
    D = oracle.ef_csm(gold["boti_X"], gold["boti_Y"], 1, gold["boti_C1"], gold["boti_C2"])
    np.testing.assert_allclose(D, gold["boti_cosine"], rtol=1e-5, atol=1e-5)
    assert oracle.lib().or_ef_oti(oracle._p(np.ascontiguousarray(gold["boti_C1"], np.float32), oracle._fp),
                                  oracle._p(np.ascontiguousarray(gold["boti_C2"], np.float32), oracle._fp)) == \
        npo.get_oti(gold["boti_C1"], gold["boti_C2"])


def test_ef_oti_golden(gold):
    for a, b, k in zip(gold["oti_C1"], gold["oti_C2"], gold["oti_idx"]):
        got = oracle.lib().or_ef_oti(oracle._p(np.ascontiguousarray(a, np.float32), oracle._fp),
                                     oracle._p(np.ascontiguousarray(b, np.float32), oracle._fp))
        assert got == int(k)


def test_ef_binarize_golden(gold):
    D = gold["bin_D"]
    for kappa, key in ((0.095, "bin_k0095"), (0.1, "bin_k01"), (5, "bin_k5")):
        np.testing.assert_array_equal(oracle.ef_binarize(D, kappa), gold[key])
    np.testing.assert_array_equal(oracle.ef_binarize(gold["bin_tie_D"], 3), gold["bin_tie_k3"])


def _int_blocks(rng, nb):
    return {"mfccs": rng.integers(-2, 3, size=(nb, 1000)).astype(np.float32),
            "ssms": rng.integers(0, 4, size=(nb, 1225)).astype(np.float32),
            "chromas": np.stack([np.isin(np.arange(480), rng.choice(480, 16, replace=False))
                                 for _ in range(nb)]).astype(np.float32)}


def test_ef_csm_exact_on_integer_blocks():
    rng = np.random.default_rng(11)
    a, b = _int_blocks(rng, 17), _int_blocks(rng, 23)
    for k in ("mfccs", "ssms"):
        np.testing.assert_array_equal(oracle.ef_csm(a[k], b[k], 0), npo.get_csm(a[k], b[k]))
    ma, mb = rng.random(12).astype(np.float32), rng.random(12).astype(np.float32)
    np.testing.assert_array_equal(oracle.ef_csm(a["chromas"], b["chromas"], 1, ma, mb),
                                  npo.get_csm_blocked_oti(a["chromas"], b["chromas"], ma, mb, npo.get_csm_cosine))


def test_ef_batch_equals_numpy_composition_on_integer_blocks():
    rng = np.random.default_rng(12)
    nbs = [int(v) for v in rng.integers(14, 40, size=7)]
    feats = [_int_blocks(rng, n) for n in nbs]
    med = rng.random((len(nbs), 12)).astype(np.float32)
    bank = {k: np.concatenate([f[k] for f in feats]) for k in ("mfccs", "ssms", "chromas")}
    bank["chroma_med"] = med
    bank["nb"] = np.array(nbs, np.int32)
    bank["off"] = np.concatenate([[0], np.cumsum(nbs[:-1])]).astype(np.int64)
    pairs = np.array([(i, j) for i in range(len(nbs)) for j in range(len(nbs)) if i != j], np.int32)
    got = oracle.ef_batch(bank, pairs, 0.1)
    for p, (i, j) in enumerate(pairs):
        f1, f2 = feats[i], feats[j]
        C = [npo.get_csm(f1["mfccs"], f2["mfccs"]), npo.get_csm(f1["ssms"], f2["ssms"]),
             npo.get_csm_blocked_oti(f1["chromas"], f2["chromas"], med[i], med[j], npo.get_csm_cosine)]
        ref = [oracle.sw_constrained(npo.csm_to_binary(M, 0.1)) for M in C]
        assert list(got[p, :3]) == ref, (i, j, got[p], ref)


# ---- the early score (VERDICT r05 missing #1): getWCSM x 3, their sum, exp, binarise, SW ----

def _kmean_sorted(D, k, axis):
    """Mean of the k smallest along `axis`, added one at a time in ascending order in float32 (the
    canonical order of ef_oracle.cpp / common.hpp kmean_canon)."""
    s = np.sort(np.moveaxis(np.asarray(D, np.float32), axis, -1), -1)[..., :k]
    acc = np.zeros(s.shape[:-1], np.float32)
    for t in range(k):
        acc = (acc + s[..., t]).astype(np.float32)
    return (acc / np.float32(k)).astype(np.float32)


def _wcsm_canonical_numpy(D, k1, k2, mu=0.5):
    """getWCSM (similarity_fusion.py:38-54) with the means in ascending order and exp correctly
    rounded (float64 exp rounded to float32): an independent numpy statement of or_ef_wcsm."""
    D = np.asarray(D, np.float32)
    rm, cm = _kmean_sorted(D, k2, 1), _kmean_sorted(D, k1, 0)
    eps = ((rm[:, None] + cm[None, :]) + D) / np.float32(3)
    me = np.float32(mu) * eps
    x = (-(D * D)) / (np.float32(2) * (me * me))
    return np.exp(x.astype(np.float64)).astype(np.float32)


def test_canon_expf_is_correctly_rounded_on_a_sample():
    """canon_expf (the fixed double sequence both the HIP kernels and the oracle evaluate) equals the
    correctly rounded float32 exp on every value of a seeded sample spanning the float32 range
    (numpy's own float32 exp, the reference's, is off by an ulp on about a third of them)."""
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(-110, 90, 4000), -rng.exponential(2.0, 4000), rng.uniform(-3, 0, 4000),
                        [0.0, -0.0, np.inf, -np.inf, -104.0, -103.97, 88.72, 89.0]]).astype(np.float32)
    got = oracle.canon_expf(x)
    with np.errstate(over="ignore"):
        ref = np.exp(x.astype(np.float64)).astype(np.float32)
    np.testing.assert_array_equal(got, ref)
    assert np.isnan(oracle.canon_expf(np.array([np.nan], np.float32)))[0]


def test_ef_wcsm_golden(gold):
    """or_ef_wcsm against the reference's own getWCSM output (golden): float32 tolerance (numpy's
    float32 exp and np.partition's sum order differ in the last ulps)."""
    np.testing.assert_allclose(oracle.ef_wcsm(gold["wcsm_CSM"], 10, 10), gold["wcsm_W"], rtol=1e-5, atol=1e-7)


def test_ef_wcsm_equals_canonical_numpy():
    """or_ef_wcsm == the independent numpy statement of the canonical order, bit for bit, with ties,
    k1 != k2 and ragged shapes."""
    rng = np.random.default_rng(7)
    for M, N, k1, k2 in ((50, 60, 10, 10), (17, 33, 3, 7), (64, 40, 16, 5)):
        D = np.abs(rng.standard_normal((M, N))).astype(np.float32)
        D[3, : N // 2] = D[3, 0]  # a run of ties in a row and a column
        D[: M // 2, 5] = D[0, 5]
        np.testing.assert_array_equal(oracle.ef_wcsm(D, k1, k2), _wcsm_canonical_numpy(D, k1, k2))


def test_ef_batch_early_equals_numpy_composition_on_integer_blocks():
    """The early score of or_ef_batch == sw(csm_to_binary(exp(-(W_m + W_s + W_c)), kappa)) composed
    from the golden-pinned numpy CSMs and the canonical numpy getWCSM above, on every pair; and
    the same as the reference's own composition (np_oracle.getWCSM, np.exp) on every pair whose
    early matrix is separated at the kappa-NN boundary by more than a few float32 ulps."""
    rng = np.random.default_rng(13)
    nbs = [int(v) for v in rng.integers(14, 40, size=7)]
    feats = [_int_blocks(rng, n) for n in nbs]
    med = rng.random((len(nbs), 12)).astype(np.float32)
    bank = {k: np.concatenate([f[k] for f in feats]) for k in ("mfccs", "ssms", "chromas")}
    bank["chroma_med"] = med
    bank["nb"] = np.array(nbs, np.int32)
    bank["off"] = np.concatenate([[0], np.cumsum(nbs[:-1])]).astype(np.int64)
    pairs = np.array([(i, j) for i in range(len(nbs)) for j in range(len(nbs)) if i != j], np.int32)
    got = oracle.ef_batch(bank, pairs, 0.1, K=10)
    separated = 0
    for p, (i, j) in enumerate(pairs):
        f1, f2 = feats[i], feats[j]
        C = [npo.get_csm(f1["mfccs"], f2["mfccs"]), npo.get_csm(f1["ssms"], f2["ssms"]),
             npo.get_csm_blocked_oti(f1["chromas"], f2["chromas"], med[i], med[j], npo.get_csm_cosine)]
        S = np.zeros_like(C[0])
        for M in C:
            S = (S + _wcsm_canonical_numpy(M, 10, 10)).astype(np.float32)
        E = np.exp((-S).astype(np.float64)).astype(np.float32)
        assert got[p, 3] == oracle.sw_constrained(npo.csm_to_binary(E, 0.1)), (i, j)
        Wr = np.zeros_like(C[0])
        for M in C:
            Wr += npo.getWCSM(M, 10, 10)
        Er = np.exp(-Wr)
        nn = npo.nneighbs(0.1, Er.shape[1])
        srt = np.sort(Er.astype(np.float64), 1)
        if np.min((srt[:, nn] - srt[:, nn - 1]) / np.maximum(srt[:, nn], 1e-12)) > 5e-6:
            separated += 1
            assert got[p, 3] == oracle.sw_constrained(npo.csm_to_binary(Er, 0.1)), (i, j)
    assert separated >= len(pairs) // 2
