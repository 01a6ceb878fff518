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
    on integer-exact block features: equal.
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
        assert list(got[p]) == ref, (i, j, got[p], ref)
