"""Pin the oracle (CPU, no GPU needed): restatements vs the reference's golden vectors, plus
known-answer tests for the essentia restatement (whose reference is absent: parity unpinned,
SURVEY.md §8c). The golden vectors were produced by the reference's own Python functions
(tests/golden/make_golden.py)."""
import numpy as np
import pytest

import oracle
from oracle import np_oracle as npo


@pytest.fixture(scope="module")
def gold():
    from conftest import GOLDEN
    return np.load(GOLDEN)


@pytest.fixture(scope="module", autouse=True)
def _built():
    oracle.build()


# ---------------------------------------------------------------- numpy restatements
@pytest.mark.parametrize("tag", ["csm_s", "csm_m"])
def test_np_csm(gold, tag):
    X, Y = gold[tag + "_X"], gold[tag + "_Y"]
    np.testing.assert_allclose(npo.get_csm(X, Y), gold[tag + "_euclid"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(npo.get_csm_cosine(X, Y), gold[tag + "_cosine"], rtol=1e-5, atol=1e-5)


def test_np_blocked_oti(gold):
    for kind, fn in [("euclid", npo.get_csm), ("cosine", npo.get_csm_cosine)]:
        D = npo.get_csm_blocked_oti(gold["boti_X"], gold["boti_Y"], gold["boti_C1"], gold["boti_C2"], fn)
        np.testing.assert_allclose(D, gold["boti_" + kind], rtol=1e-5, atol=1e-5)


def test_np_oti(gold):
    got = [npo.get_oti(a, b) for a, b in zip(gold["oti_C1"], gold["oti_C2"])]
    np.testing.assert_array_equal(got, gold["oti_idx"])


def test_np_binarize(gold):
    D = gold["bin_D"]
    for key, kappa in [("bin_k0095", 0.095), ("bin_k01", 0.1), ("bin_k5", 5)]:
        np.testing.assert_array_equal(npo.csm_to_binary(D, kappa), gold[key])
    np.testing.assert_array_equal(npo.csm_to_binary(D, 0), np.ones_like(D))
    np.testing.assert_array_equal(npo.csm_to_binary(gold["bin_tie_D"], 3), gold["bin_tie_k3"])


def test_np_wcsm(gold):
    np.testing.assert_allclose(npo.getWCSM(gold["wcsm_CSM"], 10, 10), gold["wcsm_W"], rtol=1e-5)


# ---------------------------------------------------------------- C oracle vs golden
def test_oracle_sw_golden(gold):
    for i in range(7):
        assert oracle.sw_constrained(gold["sw_%d_B" % i]) == float(gold["sw_%d_score" % i])


@pytest.mark.parametrize("tag", ["simple_a", "simple_b", "simple_c"])
def test_oracle_simple_golden(gold, tag):
    A, B = gold[tag + "_A"], gold[tag + "_B"]
    k = oracle.simple_oti(A, B)
    assert k == int(gold[tag + "_oti"])
    np.testing.assert_array_equal(np.roll(B, k, axis=0), gold[tag + "_Brot"])
    Brot, k2 = npo.simple_oti(A, B)
    assert k2 == k
    np.testing.assert_allclose(oracle.simple_sim(A, B, k=k), float(gold[tag + "_score"]), rtol=1e-12)
    # the same restatement on the pre-rolled reference (k = 0) sums in another bin order
    np.testing.assert_allclose(oracle.simple_sim(A, Brot), float(gold[tag + "_score"]), rtol=1e-12)


def test_oracle_sw_nonbinary():
    B = np.eye(6, dtype=np.uint8)
    B[3, 3] = 2
    assert oracle.sw_constrained(B) == -1.0


# ---------------------------------------------------------------- essentia KATs (unpinned)
def _grid(n, ones):
    C = np.zeros((n, n), np.uint8)
    for i, j in ones:
        C[i, j] = 1
    return C


@pytest.mark.parametrize("which", [0, 1])
def test_kat_align_basic(which):
    assert oracle.align(np.zeros((20, 20), np.uint8), which=which) == 0.0
    assert oracle.align(_grid(10, [(5, 5)]), which=which) == 1.0
    # the recurrence starts at i, j = 2: cells in the first two rows/columns never score in
    # serra09 (chen17 adds the intermediate cell C[i-1][j], so row 1 can reach row 2: 1 - 0.5)
    assert oracle.align(_grid(10, [(1, 5), (5, 0)]), which=which) == (0.0 if which == 0 else 0.5)
    assert oracle.align(_grid(20, [(2 + t, 2 + t) for t in range(10)]), which=which) == 10.0


def test_kat_serra09_gap_and_skip():
    # run of 5, one zero on the diagonal (gamma_open 0.5 from the 1 before it), run of 5
    ones = [(2 + t, 2 + t) for t in range(5)] + [(8 + t, 8 + t) for t in range(5)]
    assert oracle.align(_grid(16, ones)) == 9.5
    # a run that shifts by one column through the (i-2, j-1) predecessor costs nothing
    ones = [(2, 2), (3, 3), (4, 4), (6, 5), (7, 6), (8, 7)]
    assert oracle.align(_grid(12, ones)) == 6.0
    # after a run of 5 the score decays by gamma per zero cell and does not go negative
    ones = [(2 + t, 2 + t) for t in range(5)] + [(30, 30)]
    assert oracle.align(_grid(40, ones)) == 5.0


def test_kat_oti_rolled_chroma():
    rng = np.random.default_rng(3)
    X = np.abs(rng.standard_normal((300, 12))).astype(np.float32)
    for k in range(12):
        Y = np.roll(X, k, axis=1)
        s = oracle.oti(oracle.profile(X), oracle.profile(Y))
        np.testing.assert_array_equal(np.roll(Y, s, axis=1), X)


def test_kat_identical_tracks_full_path():
    rng = np.random.default_rng(4)
    X = np.abs(rng.standard_normal((120, 12))).astype(np.float32)
    r = oracle.crp_pair(X, X)
    Mp = oracle.stacked_len(120)
    assert Mp == 111
    # every stacked frame is its own nearest neighbour: the diagonal is recurrent
    assert np.all(np.diag(r["crp"]) == 1)
    assert r["qmax"] >= Mp - 2


# ---------------------------------------------------------------- feature prep (unpinned)
def test_median_downsample_shapes():
    X = np.arange(95 * 12, dtype=np.float32).reshape(95, 12)
    D = npo.median_downsample(X)
    assert D.shape == (3, 12)
    np.testing.assert_array_equal(D[0], np.median(X[:40], 0))
    np.testing.assert_array_equal(D[2], np.median(X[80:], 0))


def test_simple_features_unit_columns():
    rng = np.random.default_rng(5)
    X = np.abs(rng.standard_normal((2050, 12))).astype(np.float32)
    F = npo.simple_features(X)
    assert F.shape == (12, 20)
    np.testing.assert_allclose(np.linalg.norm(F, axis=0), 1.0, rtol=1e-12)


def test_np_snf_fused(gold):
    """The SNF step restatement (np_oracle.snf_step, the checker of acoss_snf_step), iterated with
    the reference's list aliasing, reproduces the reference's doSimilarityFusion output bit for bit."""
    fused = npo.snf_fused(list(gold["snf_D"]), K=5, niters=5, reg_diag=1)
    np.testing.assert_array_equal(fused, gold["snf_fused"])  # bit-exact
