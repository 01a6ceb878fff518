"""GPU parity of the acoss-side kernels (misc.hip, simple.hip) through the C-ABI.

Checked against tests/golden/reference_golden.npz (outputs of the reference Python functions,
tests/golden/make_golden.py) and against the C oracle (oracle/crp_oracle.cpp) on seeded inputs.
Tolerances: integer/binary/index outputs bit-exact; smith_waterman_constrained bit-exact (its
values are sums of +-1 and -0.7 in a fixed order); float32 CSMs vs numpy BLAS within 1e-4
relative (different GEMM summation order); SiMPle f64 vs the reference's FFT/STOMP within
1e-9 relative and bit-exact vs the oracle's direct-sum restatement.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

@pytest.fixture(scope="module")
def gold():
    from conftest import GOLDEN
    return np.load(GOLDEN)


@pytest.fixture(scope="module")
def lib():
    from acoss import _lib
    _lib.load_library()
    return _lib


def _np(t):
    return t.detach().cpu().numpy()


# ---------------------------------------------------------------- CSM (A5, A6, A2, get_ssm)
@pytest.mark.parametrize("tag", ["csm_s", "csm_m"])
@pytest.mark.parametrize("kind", ["euclid", "cosine"])
def test_csm_golden(gold, lib, tag, kind):
    X, Y = gold[tag + "_X"], gold[tag + "_Y"]
    D = _np(lib.csm(X, Y, kind=kind))
    ref = gold["%s_%s" % (tag, kind)]
    assert D.shape == ref.shape
    np.testing.assert_allclose(D, ref, rtol=1e-4, atol=1e-4 * max(1.0, float(np.abs(ref).max())))


@pytest.mark.parametrize("kind", ["euclid", "cosine"])
def test_csm_blocked_oti_golden(gold, lib, kind):
    oti = int(_np(lib.get_oti(gold["boti_C1"], gold["boti_C2"]))[0])
    D = _np(lib.csm(gold["boti_X"], gold["boti_Y"], kind=kind, oti_shift=oti))
    np.testing.assert_allclose(D, gold["boti_" + kind], rtol=1e-4, atol=2e-4)


def test_csm_large_and_ragged(lib):
    rng = np.random.default_rng(7)
    for M, N, d in [(1, 1, 1), (65, 130, 33), (257, 300, 1225), (500, 431, 480)]:
        X = rng.standard_normal((M, d)).astype(np.float32)
        Y = rng.standard_normal((N, d)).astype(np.float32)
        X64, Y64 = X.astype(np.float64), Y.astype(np.float64)
        C = (X64 ** 2).sum(1)[:, None] + (Y64 ** 2).sum(1)[None, :] - 2 * X64 @ Y64.T
        ref = np.sqrt(np.maximum(C, 0))
        D = _np(lib.csm(X, Y, kind="euclid"))
        np.testing.assert_allclose(D, ref, rtol=1e-4, atol=1e-3 * np.sqrt(d))
        Xn = X64 / np.maximum(np.linalg.norm(X64, axis=1, keepdims=True), 1e-300)
        Yn = Y64 / np.maximum(np.linalg.norm(Y64, axis=1, keepdims=True), 1e-300)
        Dc = _np(lib.csm(X, Y, kind="cosine"))
        np.testing.assert_allclose(Dc, 1 - Xn @ Yn.T, atol=2e-5)


def test_ssm_and_zero_rows(lib):
    rng = np.random.default_rng(8)
    X = rng.standard_normal((150, 1000)).astype(np.float32)
    X[3] = 0
    S = _np(lib.csm(X, kind="ssm"))
    X64 = X.astype(np.float64)
    sq = (X64 ** 2).sum(1)
    ref = np.sqrt(np.maximum(sq[:, None] + sq[None, :] - 2 * X64 @ X64.T, 0))
    np.fill_diagonal(ref, 0)
    assert np.all(np.diag(S) == 0)
    np.testing.assert_allclose(S, ref, rtol=1e-4, atol=2e-2)
    # cosine with a zero-norm row: XNorm == 0 -> 1, so the distance row is exactly 1
    Dc = _np(lib.csm(X, X, kind="cosine"))
    assert np.all(Dc[3] == 1.0) and np.all(Dc[:, 3] == 1.0)


# ---------------------------------------------------------------- get_oti (A1)
def test_get_oti_golden(gold, lib):
    idx = _np(lib.get_oti(gold["oti_C1"], gold["oti_C2"]))
    np.testing.assert_array_equal(idx, gold["oti_idx"])


# ---------------------------------------------------------------- csm_to_binary (A7)
@pytest.mark.parametrize("key,kappa", [("bin_k0095", 0.095), ("bin_k01", 0.1), ("bin_k5", 5)])
def test_binarize_golden(gold, lib, key, kappa):
    D = gold["bin_D"]
    nn = int(np.round(kappa * D.shape[1])) if kappa < 1 else int(kappa)
    B = _np(lib.binarize_rows(D, nn))
    np.testing.assert_array_equal(B, gold[key])


def test_binarize_ties_lowest_index(gold, lib):
    # the reference's argpartition picked the lowest tied columns here (2, 5, 7)
    B = _np(lib.binarize_rows(gold["bin_tie_D"], 3))
    np.testing.assert_array_equal(B, gold["bin_tie_k3"])


def test_binarize_negative_and_wide(lib):
    rng = np.random.default_rng(9)
    D = rng.standard_normal((37, 5000)).astype(np.float32)
    D[5, ::7] = -0.0
    D[6, :] = 0.0
    for nn in [1, 17, 475, 4999]:
        B = _np(lib.binarize_rows(D, nn))
        assert np.all(B.sum(1) == nn)
        for i in range(D.shape[0]):
            order = np.lexsort((np.arange(D.shape[1]), D[i]))  # value, then column
            ref = np.zeros(D.shape[1], np.uint8)
            ref[order[:nn]] = 1
            if i == 5:  # -0.0 and 0.0 are distinct keys here but equal for numpy: check counts only
                continue
            np.testing.assert_array_equal(B[i], ref)


# ---------------------------------------------------------------- getWCSM (A14)
def test_wcsm_golden(gold, lib):
    W = _np(lib.wcsm(gold["wcsm_CSM"], 10, 10, 0.5))
    np.testing.assert_allclose(W, gold["wcsm_W"], rtol=2e-4, atol=1e-7)


# ---------------------------------------------------------------- smith_waterman_constrained (A8)
def test_sw_golden(gold, lib):
    mats = [gold["sw_%d_B" % i] for i in range(7)]
    got = _np(lib.sw_constrained(mats))
    ref = np.array([float(gold["sw_%d_score" % i]) for i in range(7)])
    np.testing.assert_array_equal(got, ref)


def test_sw_vs_oracle_bands(lib):
    rng = np.random.default_rng(10)
    shapes = [(4, 4), (3, 500), (1023, 17), (1024, 40), (1025, 300), (2100, 1500), (700, 2500)]
    mats = []
    for r, c in shapes:
        p = rng.uniform(0.05, 0.5)
        B = (rng.random((r, c)) < p).astype(np.uint8)
        # plant a few diagonal runs so the maxima are large
        for _ in range(5):
            i0, j0, L = rng.integers(0, r), rng.integers(0, c), rng.integers(5, 300)
            for t in range(L):
                if i0 + t < r and j0 + t < c:
                    B[i0 + t, j0 + t] = 1
        mats.append(B)
    got = _np(lib.sw_constrained(mats))
    ref = np.array([oracle.sw_constrained(B) for B in mats])
    np.testing.assert_array_equal(got, ref)


def test_sw_nonbinary_raises(lib):
    B = np.ones((10, 10), np.uint8)
    B[4, 4] = 2
    with pytest.raises(IOError):
        lib.sw_constrained([B])
    with pytest.raises(IOError):
        lib.sw_constrained([np.full((5, 5), 0.5)])


# ---------------------------------------------------------------- SiMPle (A3, A11)
@pytest.mark.parametrize("tag", ["simple_a", "simple_b", "simple_c"])
def test_simple_golden(gold, lib, tag):
    A, B = gold[tag + "_A"], gold[tag + "_B"]
    score, oti = lib.simple_mp([A, B], np.array([[0, 1]]))
    assert int(_np(oti)[0]) == int(gold[tag + "_oti"])
    s = float(_np(score)[0])
    np.testing.assert_allclose(s, float(gold[tag + "_score"]), rtol=1e-9)
    # bit-exact against the oracle's direct-sum restatement on the rolled reference
    assert s == oracle.simple_sim(A, B, 10, k=int(gold[tag + "_oti"]))


def test_simple_batch_vs_oracle(lib):
    rng = np.random.default_rng(11)
    feats = []
    for n in [10, 11, 25, 64, 300, 257]:
        F = np.abs(rng.standard_normal((12, n)))
        F /= np.linalg.norm(F, axis=0, keepdims=True)
        feats.append(F)
    pairs = np.array([(i, j) for i in range(len(feats)) for j in range(len(feats))], dtype=np.int32)
    score, oti = lib.simple_mp(feats, pairs)
    score, oti = _np(score), _np(oti)
    for p, (i, j) in enumerate(pairs):
        k = oracle.simple_oti(feats[i], feats[j])
        assert oti[p] == k
        ref = oracle.simple_sim(feats[i], feats[j], 10, k=k)
        assert score[p] == ref or (np.isnan(ref) and np.isnan(score[p]))


@pytest.mark.parametrize("sslen,kdiag", [(10, None), (10, "mfma0"), (10, "2"), (10, "4"), (10, "5"), (7, None)])
def test_simple_long_vs_oracle(lib, monkeypatch, sslen, kdiag):
    """The MFMA kernel (the default at these lengths), the VALU diagonal kernels (ACOSS_SIMPLE_MFMA=0;
    K = 2 / 4 / 5 diagonals per lane, K = 4 passing frames by DPP) and the generic sslen path on
    tracks up to 1300 frames with unequal lengths (ragged diagonal groups), bit-exact."""
    if kdiag is not None:
        monkeypatch.setenv("ACOSS_SIMPLE_MFMA", "0")
        if kdiag != "mfma0":
            monkeypatch.setenv("ACOSS_SIMPLE_K", kdiag)
    rng = np.random.default_rng(5 + sslen)
    feats = []
    for n in [9, 10, 700, 1300, 513, 96]:
        F = np.abs(rng.standard_normal((12, n)))
        F /= np.linalg.norm(F, axis=0, keepdims=True)
        feats.append(F)
    feats.append(feats[2].copy())  # identical tracks: zero distances
    pairs = np.array([(i, j) for i in range(len(feats)) for j in range(len(feats)) if (i + j) % 2 == 0 or i == 6],
                     dtype=np.int32)
    score, oti = lib.simple_mp(feats, pairs, sslen=sslen)
    score, oti = _np(score), _np(oti)
    for p, (i, j) in enumerate(pairs):
        k = oracle.simple_oti(feats[i], feats[j])
        assert oti[p] == k
        ref = oracle.simple_sim(feats[i], feats[j], sslen, k=k)
        assert score[p] == ref or (np.isnan(ref) and np.isnan(score[p])), (i, j, score[p], ref)


@pytest.mark.parametrize("mfma", ["1", "0"])
def test_simple_max_length_vs_oracle(lib, monkeypatch, mfma):
    """A 4096-frame track (the ABI's maximum: 64 KB of per-pair LDS in the VALU kernel, 32 KB of
    sort keys in the MFMA one) against a short one, both directions, plus the short track against
    itself (zero distances); bit-exact against the oracle on both kernels."""
    monkeypatch.setenv("ACOSS_SIMPLE_MFMA", mfma)
    rng = np.random.default_rng(4096)
    feats = []
    for n in [4096, 350]:
        F = np.abs(rng.standard_normal((12, n)))
        F /= np.linalg.norm(F, axis=0, keepdims=True)
        feats.append(F)
    pairs = np.array([(0, 1), (1, 0), (1, 1)], dtype=np.int32)
    score, oti = lib.simple_mp(feats, pairs)
    score, oti = _np(score), _np(oti)
    for p, (i, j) in enumerate(pairs):
        k = oracle.simple_oti(feats[i], feats[j])
        assert oti[p] == k
        assert score[p] == oracle.simple_sim(feats[i], feats[j], 10, k=k), (i, j)


@pytest.mark.parametrize("env", [
    {"ACOSS_SIMPLE_SH": "0"},                                        # K = 4 without frame passing
    {"ACOSS_SIMPLE_PPB": "2"},                                       # 2 pairs per block
    {"ACOSS_SIMPLE_K": "4", "ACOSS_SIMPLE_SH": "0", "ACOSS_SIMPLE_PPB": "2", "ACOSS_SIMPLE_RED": "1"},
    {"ACOSS_SIMPLE_K": "2", "ACOSS_SIMPLE_RED": "1"},                # LDS row-minimum chunks
    {"ACOSS_SIMPLE_K": "0"},                                         # invalid overrides fall back to the default
    {"ACOSS_SIMPLE_K": "junk", "ACOSS_SIMPLE_PPB": "3"},
    {"ACOSS_SIMPLE_MFMA": "1"},                                      # the MFMA kernel on short tracks (10..199)
])
def test_simple_kernel_variants_vs_oracle(lib, monkeypatch, env):
    """Every SiMPle kernel variant reachable through the overrides, on short ragged tracks, bit-exact;
    the pairs name only some of the tracks (per-track scratch is built for those alone)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(17)
    feats = []
    for n in [40, 12, 150, 199, 10, 77, 130, 64]:
        F = np.abs(rng.standard_normal((12, n)))
        F /= np.linalg.norm(F, axis=0, keepdims=True)
        feats.append(F)
    used = [0, 2, 3, 5, 6]
    pairs = np.array([(i, j) for i in used for j in used], dtype=np.int32)
    score, oti = lib.simple_mp(feats, pairs)
    score, oti = _np(score), _np(oti)
    for p, (i, j) in enumerate(pairs):
        k = oracle.simple_oti(feats[i], feats[j])
        assert oti[p] == k
        assert score[p] == oracle.simple_sim(feats[i], feats[j], 10, k=k), (i, j, env)
