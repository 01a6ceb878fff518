"""GPU tests of the plugin layer: feature-prep kernels, SNF, and end-to-end
coverid.benchmark runs on synthetic on-disk datasets, each checked against the oracle.

Bars: median downsample bit-exact (same float32 arithmetic as np.median); SiMPle features
within 1e-12 relative of the numpy restatement (convolution order); Serra09/Chen Ds
bit-exact vs oracle.crp_batch on the oracle's own features, after the reference's
symmetrisation and length normalisation; SiMPle Ds bit-exact vs the C oracle on the GPU's
features; SNF within 1e-9 of the reference's golden output; EarlyFusion's composition
checked per stage (CSM tolerance, SW exact on the produced binary matrices)."""
import numpy as np
import pytest

import oracle
from oracle import np_oracle as npo
from acoss import _lib, synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gold():
    from conftest import GOLDEN
    return np.load(GOLDEN)


def _tracks(lengths, seed=3):
    rng = np.random.default_rng(seed)
    return [np.abs(rng.standard_normal((n, 12))).astype(np.float32) for n in lengths]


def test_median_downsample_bitexact():
    tr = _tracks([1, 39, 40, 41, 80, 1999, 2000, 2401])
    tr[3][5:9] = 0.25  # ties inside a segment
    feats, off, lens = synthetic.pack(tr)
    out, out_off, out_len = _lib.median_downsample(feats, off, lens, 40)
    host = out.cpu().numpy()
    for t, o, n in zip(tr, out_off, out_len):
        np.testing.assert_array_equal(host[o:o + n], npo.median_downsample(t, 40))


def test_simple_features_match_restatement():
    tr = _tracks([100, 250, 2000, 2099, 5123])
    feats, off, lens = synthetic.pack(tr)
    out, out_off, T = _lib.simple_features(feats, off, lens)
    host = out.cpu().numpy()
    for t, o, n in zip(tr, out_off, T):
        ref = npo.simple_features(t)
        got = host[o:o + 12 * n].reshape(12, n)
        np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-15)


def test_snf_golden(gold):
    from acoss.algorithms.utils.similarity_fusion import doSimilarityFusion
    Ws, fused = doSimilarityFusion(list(gold["snf_D"]), K=5, niters=5, reg_diag=1)
    np.testing.assert_allclose(fused, gold["snf_fused"], rtol=1e-9, atol=1e-12)


def _dataset(tmp_path, frames=2400, mfcc=False, n_cliques=None):
    tracks, labels = synthetic.make_corpus("covers80", frames=frames, seed=11)
    keep = np.flatnonzero(labels < (n_cliques or 8))
    tracks = [tracks[k] for k in keep]
    labels = labels[keep]
    csv, fdir = synthetic.write_feature_dataset(str(tmp_path), tracks, labels, with_mfcc=mfcc)
    return csv, fdir, tracks, labels


def _oracle_crp_D(tracks, dmax=False):
    ds = [npo.median_downsample(t, 40) for t in tracks]
    feats, off, lens = synthetic.pack(ds)
    n = len(ds)
    pairs = np.array([(i, j) for i in range(n) for j in range(i + 1, n)], np.int32)
    q, d, _ = oracle.crp_batch(feats, off, lens, pairs, dmax=dmax)
    out = []
    for v in ([q, d] if dmax else [q]):
        D = np.zeros((n, n), np.float32)
        D[pairs[:, 0], pairs[:, 1]] = v
        D += D.T
        out.append(D)
    return out, np.array([len(x) for x in ds])


def test_benchmark_serra09_matches_oracle(tmp_path, monkeypatch):
    from acoss import coverid, evaluation
    monkeypatch.chdir(tmp_path)
    csv, fdir, tracks, labels = _dataset(tmp_path)
    algo = coverid.benchmark(csv, fdir, algorithm="Serra09", shortname="t", cachedir=str(tmp_path / "cache"))
    (D,), lens = _oracle_crp_D(tracks)
    D = (D / np.sqrt(lens.astype(np.float64))[None, :]).astype(np.float32)
    got = np.asarray(algo.Ds["main"])
    np.testing.assert_array_equal(got, D)
    ref_stats = evaluation.eval_statistics(D, labels)
    assert algo.getEvalStatistics("main")[3] == ref_stats[3]


# SNF tolerance on float32 inputs: W, P and S come out of float32 reductions (kNN mean, row
# sums, kNN weight sums) whose summation order differs from numpy's partition/pairwise order,
# so they differ from the reference by a few float32 ulps; 20 diffusion steps in float64 keep
# that at the 1e-6 relative level. The bar below is 1e-5 relative (plus 1e-9 absolute).
SNF_F32_RTOL = 1e-5
SNF_F32_ATOL = 1e-9


def _assert_snf_close(got, ref):
    assert got.shape == ref.shape and got.dtype == np.float64
    np.testing.assert_allclose(got, ref, rtol=SNF_F32_RTOL, atol=SNF_F32_ATOL)


def test_benchmark_chen_matches_oracle(tmp_path, monkeypatch):
    from acoss.algorithms.latefusion_chen import ChenFusion
    monkeypatch.chdir(tmp_path)
    csv, fdir, tracks, labels = _dataset(tmp_path, n_cliques=12)  # SNF K=20 needs > 21 songs
    a = ChenFusion(csv, fdir, shortname="t", cachedir=str(tmp_path / "cache"))
    a.all_pairwise(symmetric=True)
    (Q, Dm), lens = _oracle_crp_D(tracks, dmax=True)
    np.testing.assert_array_equal(np.asarray(a.Ds["qmax"]), Q)
    np.testing.assert_array_equal(np.asarray(a.Ds["dmax"]), Dm)
    with np.errstate(divide="ignore"):
        a.normalize_by_length()
        norm = np.sqrt(lens.astype(np.float64))[None, :]
        np.testing.assert_array_equal(np.asarray(a.Ds["qmax"]), (norm / Q).astype(np.float32))
    # late fusion on the normalised float32 matrices exactly as the reference leaves them,
    # inf diagonal included (getW's fill_diagonal removes it), vs the numpy restatement
    # (bit-exact vs the reference's golden doSimilarityFusion in float64)
    ins = [np.array(a.Ds[k]) for k in a.Ds]
    assert all(np.isinf(np.diag(m)).all() for m in ins)
    with np.errstate(divide="ignore", invalid="ignore"):
        ref = npo.snf_fused(ins, K=20, niters=20, reg_diag=1)
    a.do_late_fusion()
    _assert_snf_close(np.asarray(a.Ds["Late"]), ref)
    np.testing.assert_array_equal(np.asarray(a.Ds["qmax"]), -ins[0])


def test_benchmark_simple_matches_oracle(tmp_path, monkeypatch):
    from acoss import coverid
    monkeypatch.chdir(tmp_path)
    csv, fdir, tracks, labels = _dataset(tmp_path, frames=3000, n_cliques=5)
    algo = coverid.benchmark(csv, fdir, algorithm="SiMPle", shortname="t", cachedir=str(tmp_path / "cache"))
    # the GPU's own features (bit-identical input) through the C oracle
    feats = [algo.all_feats[i] for i in range(algo.N)]
    n = len(feats)
    D = np.zeros((n, n), np.float32)
    for i in range(n):
        np.testing.assert_allclose(feats[i], npo.simple_features(tracks[i]), rtol=1e-12, atol=1e-15)
        for j in range(n):
            if i != j:
                k = oracle.simple_oti(feats[i], feats[j])
                D[i, j] = -oracle.simple_sim(feats[i], feats[j], k=k)
    np.testing.assert_array_equal(np.asarray(algo.Ds["main"]), D)


def test_earlyfusion_composition(tmp_path, monkeypatch):
    from acoss.algorithms.earlyfusion_traile import EarlyFusion
    monkeypatch.chdir(tmp_path)
    csv, fdir, tracks, labels = _dataset(tmp_path, frames=3000, mfcc=True, n_cliques=12)
    ef = EarlyFusion(csv, fdir, shortname="t", cachedir=str(tmp_path / "cache"))
    ef.all_pairwise(symmetric=True)
    # the block-feature disk cache (written on a background thread, flushed by all_pairwise):
    # every song's file is there and reads back to the arrays in memory
    from acoss.features_io import load_features
    for i in range(ef.N):
        cached = load_features("%s_%i.h5" % (ef.get_cacheprefix(), i))
        for k in ("mfccs", "ssms", "chromas", "chroma_med"):
            np.testing.assert_array_equal(np.asarray(cached[k]), np.asarray(ef.all_block_feats[i][k]))
    for (i, j) in [(0, 1), (1, 4), (2, 3)]:
        f1, f2 = ef.load_features(i), ef.load_features(j)
        mats = [m.cpu().numpy() for m in ef.pair_matrices(i, j)]
        C = npo.get_csm(f1["mfccs"], f2["mfccs"])
        B = npo.csm_to_binary(C, ef.kappa)
        assert np.mean(B != mats[0]) < 0.01
        Cc = npo.get_csm_blocked_oti(f1["chromas"], f2["chromas"], f1["chroma_med"], f2["chroma_med"],
                                     npo.get_csm_cosine)
        assert np.mean(npo.csm_to_binary(Cc, ef.kappa) != mats[2]) < 0.01
        Wref = sum(npo.getWCSM(c, ef.K, ef.K) for c in (C, npo.get_csm(f1["ssms"], f2["ssms"]), Cc))
        assert np.mean(npo.csm_to_binary(np.exp(-Wref), ef.kappa) != mats[3]) < 0.02
    # the batched C-ABI path (acoss_earlyfusion) equals the per-pair composition on every pair
    for i in range(ef.N):
        for j in range(i + 1, ef.N):
            mats = [m.cpu().numpy() for m in ef.pair_matrices(i, j)]
            for s, key in enumerate(["mfccs", "ssms", "chromas", "early"]):
                ref = oracle.sw_constrained(mats[s])
                assert ef.Ds[key][i, j] == np.float32(ref), (i, j, key)  # Ds is float32, like the memmap
    ins = {s: np.array(ef.Ds[s]) for s in ["chromas", "ssms", "mfccs", "early"]}
    ef.do_late_fusion()
    ref_late = npo.snf_fused([1.0 / (1.0 + ins[s]) for s in ["chromas", "ssms", "mfccs"]], K=20, niters=20)
    ref_el = npo.snf_fused([1.0 / (1.0 + ins[s]) for s in ["chromas", "ssms", "mfccs", "early"]], K=20, niters=20)
    _assert_snf_close(np.asarray(ef.Ds["late"]), ref_late)
    _assert_snf_close(np.asarray(ef.Ds["early+late"]), ref_el)


@pytest.mark.parametrize("n,K,L,vw", [(40, 5, 2, None), (333, 20, 3, None), (1030, 7, 4, None), (1030, 7, 2, "1")])
def test_snf_step_bitexact(monkeypatch, n, K, L, vw):
    """acoss_snf_step vs the reference's own scipy expression (np_oracle.snf_step): the HIP
    kernels sum in csr column order with unfused multiply/add, so the result is bit-exact.
    Even n gathers two columns per lane (16-byte loads), odd n one; vw = "1" forces one."""
    import torch
    if vw:
        monkeypatch.setenv("ACOSS_SNF_VW", vw)
    rng = np.random.default_rng(n)
    mats = [rng.random((n, n)) for _ in range(L)]
    J = np.stack([rng.choice(n, K, replace=False) for _ in range(n)]).astype(np.int32)
    V = rng.random((n, K)).astype(np.float32)
    V = (V / V.sum(1, keepdims=True)).astype(np.float64)
    dm = [torch.as_tensor(m).cuda() for m in mats]
    for skip in range(L):
        got = _lib.snf_step(dm, skip, J, V, 1.0).cpu().numpy()
        np.testing.assert_array_equal(got, npo.snf_step(mats, skip, J, V, 1.0))
    got = _lib.snf_step(dm, 0, J, V, 0.0).cpu().numpy()
    np.testing.assert_array_equal(got, npo.snf_step(mats, 0, J, V, 0.0))


def test_snf_step_many_matrices():
    """More matrices than one kernel-argument chunk (16): the average runs in passes and stays
    bit-exact (same ascending summation order)."""
    import torch
    n, K, L = 70, 6, 37
    rng = np.random.default_rng(7)
    mats = [rng.random((n, n)) for _ in range(L)]
    J = np.stack([rng.choice(n, K, replace=False) for _ in range(n)]).astype(np.int32)
    V = rng.random((n, K))
    dm = [torch.as_tensor(m).cuda() for m in mats]
    for skip in (0, 16, 17, L - 1):
        got = _lib.snf_step(dm, skip, J, V, 1.0).cpu().numpy()
        np.testing.assert_array_equal(got, npo.snf_step(mats, skip, J, V, 1.0))


@pytest.mark.parametrize("n,K,L,world", [(40, 5, 2, 2), (333, 20, 3, 3), (1030, 7, 4, 8), (70, 6, 19, 4)])
def test_snf_rows_split_bitexact(n, K, L, world):
    """The row-sharded step (acoss_snf_diffuse_rows, gather, acoss_snf_left_rows) stripe by
    stripe equals acoss_snf_step and the scipy expression, for ragged last stripes and more
    matrices than one argument chunk."""
    import torch
    from acoss.algorithms.utils.similarity_fusion import shard_rows
    rng = np.random.default_rng(n + L)
    mats = [rng.random((n, n)) for _ in range(L)]
    J = np.stack([rng.choice(n, K, replace=False) for _ in range(n)]).astype(np.int32)
    V = rng.random((n, K))
    dm = [torch.as_tensor(m).cuda() for m in mats]
    bounds = shard_rows(n, world)
    for skip in sorted({0, L - 1}):
        ref = npo.snf_step(mats, skip, J, V, 1.0)
        Bs = [_lib.snf_diffuse_rows([m[r0:r1].contiguous() for m in dm], skip, n, J, V) for r0, r1 in bounds]
        B = torch.cat(Bs, 0).contiguous()
        got = torch.cat([_lib.snf_left_rows(B, r0, r1 - r0, J, V, 1.0) for r0, r1 in bounds], 0).cpu().numpy()
        np.testing.assert_array_equal(got, ref)
        np.testing.assert_array_equal(_lib.snf_step(dm, skip, J, V, 1.0).cpu().numpy(), ref)
    # the output stripe may reuse the skipped matrix's stripe; other overlaps are refused
    st = [m[:7].contiguous() for m in dm]
    want = _lib.snf_diffuse_rows(st, 0, n, J, V).clone()
    np.testing.assert_array_equal(_lib.snf_diffuse_rows(st, 0, n, J, V, out=st[0]).cpu().numpy(), want.cpu().numpy())
    with pytest.raises(_lib.AcossHipError):
        _lib.snf_diffuse_rows(st, 0, n, J, V, out=st[1])
    B = torch.zeros((n, n), dtype=torch.float64, device="cuda")
    with pytest.raises(_lib.AcossHipError):
        _lib.snf_left_rows(B, 0, 3, J, V, 1.0, out=B[5:8])
    with pytest.raises(_lib.AcossHipError):
        _lib.snf_left_rows(B, n - 2, 3, J, V, 1.0)


def test_snf_float32_matches_restatement():
    """doSimilarityFusion on float32 distance matrices (the ChenFusion / EarlyFusion input dtype)
    vs the numpy restatement at the stated SNF tolerance, with an inf diagonal as Chen has."""
    from acoss.algorithms.utils.similarity_fusion import doSimilarityFusion
    rng = np.random.default_rng(5)
    n = 150
    Ds = []
    for _ in range(3):
        D = (rng.random((n, n)) * 10 + 0.5).astype(np.float32)
        np.fill_diagonal(D, np.inf)
        Ds.append(D)
    Ws, fused = doSimilarityFusion(Ds, K=20, niters=20, reg_diag=1)
    with np.errstate(invalid="ignore"):
        ref = npo.snf_fused(Ds, K=20, niters=20, reg_diag=1)
    assert Ws[0].dtype == np.float32
    _assert_snf_close(fused, ref)


def test_snf_single_matrix_is_nan():
    """One matrix: the reference divides the empty average by N - 1 = 0, so every entry is nan."""
    from acoss.algorithms.utils.similarity_fusion import doSimilarityFusionWs
    W = np.random.default_rng(1).random((12, 12))
    with pytest.warns(RuntimeWarning):
        F = doSimilarityFusionWs([W], K=3, niters=2)
    assert F.shape == (12, 12) and np.isnan(F).all()


def test_snf_step_rejects_bad_args():
    import ctypes
    import torch
    m = torch.zeros((8, 8), dtype=torch.float64, device="cuda")
    J = np.tile(np.arange(2, dtype=np.int32), (8, 1))
    V = np.zeros((8, 2))
    with pytest.raises(ValueError):
        _lib.snf_step([m], 0, J, V, 1.0)  # one matrix: nothing to average
    with pytest.raises(ValueError):
        _lib.snf_step([m, m.float()], 0, J, V, 1.0)
    for bad in (8, -1):  # column outside [0, n)
        Jb = J.copy()
        Jb[3, 1] = bad
        with pytest.raises(ValueError):
            _lib.snf_step([m, m.clone()], 0, Jb, V, 1.0)
    Jd = J.copy()
    Jd[5] = [4, 4]  # repeated column in a row
    with pytest.raises(ValueError):
        _lib.snf_step([m, m.clone()], 0, Jd, V, 1.0)
    # the C-ABI checks the same on the device (a caller that skips the Python wrapper)
    lib = _lib.load_library()
    m2 = m.clone()
    out = torch.empty_like(m)
    ptrs = (ctypes.c_void_p * 2)(m.data_ptr(), m2.data_ptr())
    Vd = torch.as_tensor(V).cuda()
    for Jbad in (Jb, Jd, np.full((8, 2), 1 << 20, np.int32)):
        Jt = torch.as_tensor(Jbad).cuda()
        rc = lib.acoss_snf_step(ptrs, 2, 0, 8, ctypes.c_void_p(Jt.data_ptr()), ctypes.c_void_p(Vd.data_ptr()), 2,
                                1.0, ctypes.c_void_p(out.data_ptr()), 1, _lib._stream())
        assert rc == -1 and b"kNN column" in lib.acoss_last_error()
        # unvalidated: no error code, and the bad row is harmless (no read outside the matrices)
        rc = lib.acoss_snf_step(ptrs, 2, 0, 8, ctypes.c_void_p(Jt.data_ptr()), ctypes.c_void_p(Vd.data_ptr()), 2,
                                1.0, ctypes.c_void_p(out.data_ptr()), 0, _lib._stream())
        assert rc == 0
        torch.cuda.synchronize()
    Jt = torch.as_tensor(J).cuda()
    rc = lib.acoss_snf_step(ptrs, 2, 0, 8, ctypes.c_void_p(Jt.data_ptr()), ctypes.c_void_p(Vd.data_ptr()), 2, 1.0,
                            ctypes.c_void_p(out.data_ptr()), 1, _lib._stream())
    assert rc == 0
