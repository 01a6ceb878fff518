"""EarlyFusion end to end against the numpy oracle composition (A15, GPU).

EarlyFusion.similarity (acoss/algorithms/earlyfusion_traile.py:157-198) composes three CSMs
(float32 BLAS in the reference, MFMA here), a kappa-NN row binarisation, getWCSM and four
constrained Smith-Waterman alignments. In general the CSMs of the two paths differ in float32
summation order, so a row whose kappa-th and (kappa+1)-th smallest values are within a few ulps
could binarise differently. The block features here are built so that every CSM is EXACT in
any summation order: small-integer MFCC / SSM blocks (every |x|^2, x.y and d^2 is an integer
below 2^24; sqrt correctly rounded on both sides) and 0/1 chroma blocks with exactly 16 ones
(norm 4, so the normalised rows and their dot products are exact binary fractions). Both paths
then see bit-identical CSMs, resolve ties by the same lowest-column rule (acoss_binarize_rows,
np_oracle.csm_to_binary), and the three per-feature scores must be EQUAL to the oracle's.

The early-fusion matrix exp(-sum getWCSM) follows the canonical order of oracle/ef_oracle.cpp
(the k smallest summed ascending, exp = canon_expf), so the early score is EQUAL to that oracle on
EVERY pair (the oracle is pinned in tests/test_ef_oracle.py against the golden getWCSM and an
independent numpy statement). Against the reference's own composition (numpy's np.partition
order and float32 exp) it is asserted equal on every pair whose early matrix is separated at the
kappa-NN boundary by more than EARLY_MARGIN relative, at least 70 % of the pairs. The late /
early+late SNF outputs (:200-206) must match np_oracle.snf_fused of the ORACLE's matrices at the
SNF float32 tolerance of test_gpu_plugin.py.
"""
import numpy as np
import pytest

import oracle
from oracle import np_oracle as npo
from acoss import synthetic

pytestmark = pytest.mark.gpu

N_TRACKS = 24          # SNF with K = 20 needs more than 21 songs
EARLY_MARGIN = 5e-6   # ~5x the float32 error of the getWCSM mean / exp chain


def _clique_blocks(rng, nb):
    """Integer-exact block features of one clique's base song."""
    return {"mfccs": rng.integers(-2, 3, size=(nb, 1000)).astype(np.float32),
            "ssms": rng.integers(0, 4, size=(nb, 1225)).astype(np.float32),
            "chromas": _chroma_rows(rng, nb)}


def _chroma_rows(rng, nb):
    X = np.zeros((nb, 480), np.float32)
    for b in range(nb):
        X[b, rng.choice(480, 16, replace=False)] = 1.0
    return X


def _cover(rng, base, nb):
    """A cover: the base's blocks from a random start, resampled to nb blocks, with integer
    perturbations (still exact) and a few chroma ones moved."""
    n0 = len(base["mfccs"])
    idx = np.minimum((np.arange(nb) * (n0 / nb) + rng.integers(0, 5)).astype(np.int64), n0 - 1)
    out = {}
    out["mfccs"] = np.clip(base["mfccs"][idx] + rng.integers(-1, 2, size=(nb, 1000)) * (rng.random((nb, 1000)) < 0.3),
                           -2, 2).astype(np.float32)
    out["ssms"] = np.clip(base["ssms"][idx] + rng.integers(-1, 2, size=(nb, 1225)) * (rng.random((nb, 1225)) < 0.3),
                          0, 3).astype(np.float32)
    ch = base["chromas"][idx].copy()
    for b in range(nb):
        if rng.random() < 0.5:
            on, off = np.flatnonzero(ch[b] == 1), np.flatnonzero(ch[b] == 0)
            ch[b, rng.choice(on, 4, replace=False)] = 0
            ch[b, rng.choice(off, 4, replace=False)] = 1
    out["chromas"] = ch
    return out


def _boundary_margin(D, nn):
    s = np.sort(D.astype(np.float64), 1)
    gap = s[:, nn] - s[:, nn - 1]
    return float(np.min(gap / np.maximum(np.abs(s[:, nn]), 1e-12)))


def _oracle_pair(f1, f2, kappa, K):
    C = {"mfccs": npo.get_csm(f1["mfccs"], f2["mfccs"]), "ssms": npo.get_csm(f1["ssms"], f2["ssms"]),
         "chromas": npo.get_csm_blocked_oti(f1["chromas"], f2["chromas"], f1["chroma_med"], f2["chroma_med"],
                                           npo.get_csm_cosine)}
    W = np.zeros_like(C["mfccs"])
    for s in ("mfccs", "ssms", "chromas"):
        W += npo.getWCSM(C[s], K, K)
    E = np.exp(-W)
    mats = [C["mfccs"], C["ssms"], C["chromas"], E]
    return mats, [oracle.sw_constrained(npo.csm_to_binary(M, kappa)) for M in mats]


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    root = tmp_path_factory.mktemp("efpin")
    rng = np.random.Generator(np.random.PCG64(2024))
    feats, labels = [], []
    for c in range(N_TRACKS // 2):
        base = _clique_blocks(rng, int(rng.integers(40, 90)))
        for v in range(2):
            bf = dict(base) if v == 0 else _cover(rng, base, int(rng.integers(40, 90)))
            # integer medians (exact in float32): the blocked-OTI roll varies by pair
            bf["chroma_med"] = rng.permutation(12).astype(np.float32)
            feats.append(bf)
            labels.append(c)
    # per-track input files only carry the clique labels; the block features go straight into
    # the plugin's per-track cache ('<prefix>_<i>.h5' -> .npz twin), as load_features reads them
    tracks = [np.zeros((8, 12), np.float32) for _ in range(N_TRACKS)]
    csv, fdir = synthetic.write_feature_dataset(str(root), tracks, np.asarray(labels))
    return root, csv, fdir, feats


def test_earlyfusion_scores_equal_oracle(corpus, monkeypatch):
    from acoss.algorithms.earlyfusion_traile import EarlyFusion
    from acoss.features_io import save_features
    root, csv, fdir, feats = corpus
    monkeypatch.chdir(root)
    ef = EarlyFusion(csv, fdir, shortname="pin", cachedir=str(root / "cache"))
    for i, bf in enumerate(feats):
        save_features("%s_%i.h5" % (ef.get_cacheprefix(), i), bf)
    ef.all_pairwise(symmetric=True)
    keys = ["mfccs", "ssms", "chromas", "early"]
    ref = {k: np.zeros((N_TRACKS, N_TRACKS), np.float32) for k in keys}
    safe = np.zeros((N_TRACKS, N_TRACKS), bool)
    otis = set()
    for i in range(N_TRACKS):
        for j in range(i + 1, N_TRACKS):
            mats, scores = _oracle_pair(feats[i], feats[j], ef.kappa, ef.K)
            nn = npo.nneighbs(ef.kappa, mats[0].shape[1])
            safe[i, j] = safe[j, i] = _boundary_margin(mats[3], nn) > EARLY_MARGIN
            otis.add(npo.get_oti(feats[i]["chroma_med"], feats[j]["chroma_med"]))
            for k, v in zip(keys, scores):
                ref[k][i, j] = v
    assert len(otis) >= 6  # the roll is exercised
    npairs = N_TRACKS * (N_TRACKS - 1) // 2
    assert np.triu(safe, 1).sum() >= 0.7 * npairs
    # the canonical-order oracle on every pair, all four scores
    nbs = [len(f["mfccs"]) for f in feats]
    bank = {k: np.concatenate([f[k] for f in feats]) for k in ("mfccs", "ssms", "chromas")}
    bank["chroma_med"] = np.stack([f["chroma_med"] for f in feats])
    bank["nb"] = np.array(nbs, np.int32)
    bank["off"] = np.concatenate([[0], np.cumsum(nbs[:-1])]).astype(np.int64)
    up = np.array([(i, j) for i in range(N_TRACKS) for j in range(i + 1, N_TRACKS)], np.int32)
    canon = oracle.ef_batch(bank, up, ef.kappa, K=ef.K)
    for k in keys:
        ref[k] += ref[k].T
        assert np.count_nonzero(ref[k]) > npairs
        got = np.asarray(ef.Ds[k])
        np.testing.assert_array_equal(got[up[:, 0], up[:, 1]], canon[:, keys.index(k)].astype(np.float32),
                                      err_msg=k + " vs the canonical oracle")
        if k == "early":
            np.testing.assert_array_equal(got[safe], ref[k][safe], err_msg=k)
        else:
            np.testing.assert_array_equal(got, ref[k], err_msg=k)
    # covers score above non-covers (the inputs carry real structure)
    lab = np.arange(N_TRACKS) // 2
    same = (lab[:, None] == lab[None, :]) & ~np.eye(N_TRACKS, dtype=bool)
    assert ref["mfccs"][same].mean() > 2 * ref["mfccs"][~same & ~np.eye(N_TRACKS, dtype=bool)].mean()
    # late fusion of the ORACLE's matrices (not the GPU's) at the SNF float32 tolerance; early+late
    # takes the GPU's early matrix (equal to the oracle's on the separated pairs) with the
    # oracle's three others
    early_gpu = np.array(ef.Ds["early"])
    late = npo.snf_fused([1.0 / (1.0 + ref[s]) for s in ["chromas", "ssms", "mfccs"]], K=20, niters=20)
    el = npo.snf_fused([1.0 / (1.0 + m) for m in (ref["chromas"], ref["ssms"], ref["mfccs"], early_gpu)], K=20,
                       niters=20)
    ef.do_late_fusion()
    np.testing.assert_allclose(np.asarray(ef.Ds["late"]), late, rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(np.asarray(ef.Ds["early+late"]), el, rtol=1e-5, atol=1e-9)


def test_ef_block_features_gpu_vs_restatement():
    """acoss_ef_block_features (efblocks.hip) vs np_oracle.ef_block_features (the reference's block
    loops with scipy's resize), ragged tracks and beat grids in one launch. Both compute in float64
    (different summation orders: the Gaussian weights' sum, the means, the SSM dots) and store
    float32, so outputs agree within one float32 rounding: |diff| <= 2e-7 * |value| + 1e-7 and
    at least 99 % of the values bit-identical. The medians are exact."""
    from acoss import _lib
    rng = np.random.default_rng(12)
    chromas, mfccs, onsets = [], [], []
    # (16000, 700): beat blocks of ~14,000 frames, Gaussian radii past the LDS tap table (on-the-fly taps)
    # (n, period, MFCC frames short of the chroma): the extractor's mfcc_htk is ~43 frames shorter
    # (acoss/features.py:884), so the last beat blocks' MFCC spans are clamped by the slicing
    # (resize_block's X[i1:i2]); (1200, 5, 100) cuts the last 20 blocks' MFCC spans short, the
    # last one to 5 frames; "dup" repeats onsets (np.round of close beats), which the reference
    # accepts while every block spans frames
    for n, period, short in [(900, 43, 0), (2601, 37, 43), (500, 11, 43), (4001, 60, 0), (860, 43, 43),
                             (16000, 700, 43), (1200, 5, 100)]:
        chromas.append(np.abs(rng.normal(size=(n, 12))).astype(np.float32))
        m = rng.normal(size=(20, n - short)).astype(np.float32)
        m[1, 5] = np.nan
        mfccs.append(m)
        o = np.arange(0, n - 1, period) + rng.integers(0, 4, size=len(range(0, n - 1, period)))
        onsets.append(np.unique(np.clip(o, 0, n - 1)).astype(np.int64))
    dup = onsets[2].copy()
    dup[10:14] = dup[10]  # four equal onsets inside a 20-beat block
    onsets[2] = np.sort(dup)
    assert onsets[6][-21] < mfccs[6].shape[1] < onsets[6][-2]  # the last blocks' spans end past the MFCC
    out = _lib.ef_block_features(chromas, [m.T for m in mfccs], onsets)
    tot, same = 0, 0
    for t in range(len(chromas)):
        ref = npo.ef_block_features(chromas[t], mfccs[t], onsets[t])
        b0, nb = int(out["block_off"][t]), int(out["n_blocks"][t])
        assert nb == max(0, len(onsets[t]) - 20)
        for key in ("mfccs", "ssms", "chromas"):
            got = out[key].cpu().numpy()[b0:b0 + nb]
            assert got.shape == ref[key].shape
            np.testing.assert_allclose(got, ref[key], rtol=2e-7, atol=1e-7, err_msg=key)
            tot += got.size
            same += int(np.sum(got == ref[key]))
        np.testing.assert_array_equal(out["chroma_med"].cpu().numpy()[t], ref["chroma_med"])
    assert same >= 0.99 * tot, (same, tot)
    # fewer beats than blocksize: the reference raises (np.zeros with a negative dimension), so does this
    short = [np.abs(rng.normal(size=(300, 12))).astype(np.float32)]
    with pytest.raises(ValueError):
        npo.ef_block_features(short[0], rng.normal(size=(20, 300)).astype(np.float32), np.arange(1, 300, 90))
    with pytest.raises(ValueError):
        _lib.ef_block_features(short, [rng.normal(size=(300, 20)).astype(np.float32)], [np.arange(1, 300, 90)])
    # a block whose MFCC span is empty after the clamp: the reference's resize raises, so does this
    ch = np.abs(rng.normal(size=(400, 12))).astype(np.float32)
    o = np.arange(0, 400, 10).astype(np.int64)
    mf = rng.normal(size=(20, 150)).astype(np.float32)  # o[20] = 200 > 150 frames of MFCC
    with pytest.raises(Exception):
        npo.ef_block_features(ch, mf, o)
    with pytest.raises(ValueError):
        _lib.ef_block_features([ch], [mf.T], [o])


_EF_KERNEL_SCRIPT = r"""
import sys, numpy as np, torch
sys.path[:0] = [sys.argv[1], sys.argv[1] + '/acoss-1_amd']
from acoss import _lib
rng = np.random.default_rng(9)
NT, NB = 7, int(sys.argv[2])
bank = {'mfccs': torch.as_tensor(rng.standard_normal((NT * NB, 1000), dtype=np.float32)).cuda(),
        'ssms': torch.as_tensor(np.abs(rng.standard_normal((NT * NB, int(sys.argv[3])), dtype=np.float32))).cuda(),
        'chromas': torch.as_tensor(np.abs(rng.standard_normal((NT * NB, 480), dtype=np.float32))).cuda(),
        'chroma_med': torch.as_tensor(np.abs(rng.standard_normal((NT, 12), dtype=np.float32))).cuda(),
        'off': torch.as_tensor(np.arange(NT, dtype=np.int64) * NB).cuda(),
        'nb': torch.as_tensor(np.full(NT, NB, np.int32)).cuda(), 'max_blocks': NB}
pairs = np.array([(i, j) for i in range(NT) for j in range(NT) if i != j], np.int32)
np.save(sys.argv[4], _lib.earlyfusion(bank, pairs, 0.1, 10).cpu().numpy())
"""


@pytest.mark.parametrize("nb,d_ssm", [(130, 1225), (64, 1000), (71, 1221)])
def test_earlyfusion_wave_csm_equals_lds_csm(tmp_path, nb, d_ssm):
    """The wave-tile CSM kernels (k_ef_csm_w: euclid, the padded SSM bank, the cosine chroma CSM
    with the OTI roll in registers) against the LDS-tiled ones (ACOSS_EF_LDS_CSM=1, read once per
    process, hence two processes): every EarlyFusion score bit-identical, over all ordered pairs
    (every OTI roll), ragged tile edges and an SSM width that is not a multiple of 4."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    out = {}
    for tag, env in (("wave", {}), ("lds", {"ACOSS_EF_LDS_CSM": "1"})):
        f = str(tmp_path / ("%s.npy" % tag))
        r = subprocess.run([sys.executable, "-c", _EF_KERNEL_SCRIPT, ROOT, str(nb), str(d_ssm), f],
                           env=dict(os.environ, **env), capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        out[tag] = np.load(f)
    assert np.isfinite(out["wave"]).all()
    np.testing.assert_array_equal(out["wave"], out["lds"])


def test_earlyfusion_scores_equal_canonical_oracle_on_float_blocks():
    """On general float32 block features (not integer-exact) the GPU's mfccs / ssms / chromas
    and early scores equal the canonical-order CPU oracle (oracle/ef_oracle.cpp, pinned against
    the reference's golden CSMs / OTI / binarisation / getWCSM in tests/test_ef_oracle.py) on every
    pair: the CSMs, the k-smallest means and exp follow the same float32 order bit for bit, and
    binarisation and SW are exact. Ragged block counts, K = 10 and K = 20 (the wave-per-line means),
    kappa = 0.1, and a kappa >= 1 count."""
    import torch
    from acoss import _lib
    rng = np.random.default_rng(31)
    nbs = [int(v) for v in rng.integers(12, 140, size=16)]
    T, R = len(nbs), sum(nbs)
    host = {"mfccs": rng.standard_normal((R, 1000), dtype=np.float32),
            "ssms": np.abs(rng.standard_normal((R, 1225), dtype=np.float32)),
            "chromas": np.abs(rng.standard_normal((R, 480), dtype=np.float32)),
            "chroma_med": np.abs(rng.standard_normal((T, 12), dtype=np.float32)),
            "nb": np.array(nbs, np.int32), "off": np.concatenate([[0], np.cumsum(nbs[:-1])]).astype(np.int64)}
    bank = {k: torch.as_tensor(host[k]).cuda() for k in ("mfccs", "ssms", "chromas", "chroma_med", "off", "nb")}
    bank["max_blocks"] = max(nbs)
    pairs = np.array([(i, j) for i in range(T) for j in range(T) if i != j], np.int32)
    for kappa, K in ((0.1, 10), (5.0, 10), (0.1, 7), (0.1, 20)):
        pk = pairs[(host["nb"][pairs[:, 0]] > K) & (host["nb"][pairs[:, 1]] > K)]  # the reference's partition bound
        got = _lib.earlyfusion(bank, pk, kappa, K).cpu().numpy()
        ref = oracle.ef_batch(host, pk, kappa, K=K)
        for f, key in enumerate(("mfccs", "ssms", "chromas", "early")):
            bad = np.flatnonzero(got[:, f] != ref[:, f])
            assert len(bad) == 0, (kappa, K, key, len(bad), pk[bad[:5]], got[bad[:5], f], ref[bad[:5], f])


_EF_SHORT_SCRIPT = r"""
import sys, numpy as np, torch
sys.path[:0] = [sys.argv[1], sys.argv[1] + '/acoss-1_amd']
from acoss import _lib
rng = np.random.default_rng(21)
NT = 96
lo, hi = (int(v) for v in sys.argv[4].split(',')) if len(sys.argv) > 4 else (14, 48)
nb = rng.integers(lo, hi, size=NT).astype(np.int32)  # Da-TACOS beat-block counts
off = np.concatenate([[0], np.cumsum(nb[:-1])]).astype(np.int64)
R = int(nb.sum())
bank = {'mfccs': torch.as_tensor(rng.standard_normal((R, 1000), dtype=np.float32)).cuda(),
        'ssms': torch.as_tensor(np.abs(rng.standard_normal((R, 1225), dtype=np.float32))).cuda(),
        'chromas': torch.as_tensor(np.abs(rng.standard_normal((R, 480), dtype=np.float32))).cuda(),
        'chroma_med': torch.as_tensor(np.abs(rng.standard_normal((NT, 12), dtype=np.float32))).cuda(),
        'off': torch.as_tensor(off).cuda(), 'nb': torch.as_tensor(nb).cuda(), 'max_blocks': int(nb.max())}
pairs = np.array([(i, j) for i in range(NT) for j in range(NT) if i != j], np.int32)
if sys.argv[3] == 'slices':  # calls of <= 4096 pairs: processed in the caller's order
    out = np.concatenate([_lib.earlyfusion(bank, pairs[k:k + 4000], 0.1, 10).cpu().numpy()
                          for k in range(0, len(pairs), 4000)])
else:  # one call of 9120 pairs: (reference band, query) order inside, scattered back
    out = _lib.earlyfusion(bank, pairs, 0.1, 10).cpu().numpy()
np.save(sys.argv[2], out)
"""


def test_earlyfusion_short_tracks_orders_and_chunks(tmp_path):
    """Da-TACOS-sized tracks (14..47 beat blocks: euclid CSM tiles with the reference columns of a
    query's run packed, cosine 32 x 32 tiles with several pairs per wave sharing their query rows,
    the row-per-lane binarize, several Smith-Waterman matrices per wave): the scores of one
    9,120-pair call (processed in (reference band, query) order and scattered back) equal those of
    4,000-pair calls in the caller's order, those of many small chunks on one stream
    (ACOSS_EF_BYTES / ACOSS_EF_STREAMS) and those of one pair per CSM wave and the 4-wave binarize
    (ACOSS_EF_W4=0, ACOSS_EF_LANEBIN=0, ACOSS_EF_PACK=0; each read once per process, hence separate
    processes), bit for bit."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    out = {}
    for tag, mode, env in (("band", "one", {}), ("slices", "slices", {}),
                           ("chunks", "one", {"ACOSS_EF_STREAMS": "1", "ACOSS_EF_BYTES": str(8 << 20)}),
                           ("w1", "one", {"ACOSS_EF_W4": "0", "ACOSS_EF_LANEBIN": "0", "ACOSS_EF_PACK": "0"}),
                           ("pack1", "one", {"ACOSS_EF_PACK": "1"})):
        f = str(tmp_path / ("%s.npy" % tag))
        r = subprocess.run([sys.executable, "-c", _EF_SHORT_SCRIPT, ROOT, f, mode],
                           env=dict(os.environ, **env), capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        out[tag] = np.load(f)
    assert np.isfinite(out["band"]).all() and out["band"].shape == (96 * 95, 4)
    np.testing.assert_array_equal(out["band"], out["slices"])
    np.testing.assert_array_equal(out["band"], out["chunks"])
    np.testing.assert_array_equal(out["band"], out["w1"])  # the short-track kernels == the one-pair-per-wave ones
    np.testing.assert_array_equal(out["band"], out["pack1"])  # 32 x 32 packed tiles
    # and all four scores of a sample of pairs == the canonical-order oracle (same bank)
    import oracle
    rng = np.random.default_rng(21)
    nb = rng.integers(14, 48, size=96).astype(np.int32)
    R = int(nb.sum())
    bank = {"mfccs": rng.standard_normal((R, 1000), dtype=np.float32),
            "ssms": np.abs(rng.standard_normal((R, 1225), dtype=np.float32)),
            "chromas": np.abs(rng.standard_normal((R, 480), dtype=np.float32)),
            "chroma_med": np.abs(rng.standard_normal((96, 12), dtype=np.float32)),
            "nb": nb, "off": np.concatenate([[0], np.cumsum(nb[:-1])]).astype(np.int64)}
    pairs = np.array([(i, j) for i in range(96) for j in range(96) if i != j], np.int32)
    idx = np.random.default_rng(3).choice(len(pairs), 150, replace=False)
    ref = oracle.ef_batch(bank, pairs[idx], 0.1)
    np.testing.assert_array_equal(out["band"][idx], np.asarray(ref, np.float64))


def test_earlyfusion_mid_tracks_packed_columns(tmp_path):
    """30..80 beat blocks (Da-TACOS songs of 350-700 chroma frames): the euclid CSMs with the
    reference columns packed into 32 x 64 tiles (k_ef_csm_pack<2>, the default up to 128 blocks)
    equal the 64 x 64 tile per pair (ACOSS_EF_PACK=0) and 32 x 32 packed tiles (ACOSS_EF_PACK=1)
    bit for bit on all four scores of every
    ordered pair (one 9,120-pair call in (reference band, query) order, separate processes), and a
    sample equals the canonical-order oracle."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    out = {}
    for tag, env in (("pack", {}), ("nopack", {"ACOSS_EF_PACK": "0"}), ("pack1", {"ACOSS_EF_PACK": "1"})):
        f = str(tmp_path / ("%s.npy" % tag))
        r = subprocess.run([sys.executable, "-c", _EF_SHORT_SCRIPT, ROOT, f, "one", "30,81"],
                           env=dict(os.environ, **env), capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        out[tag] = np.load(f)
    assert np.isfinite(out["pack"]).all()
    np.testing.assert_array_equal(out["pack"], out["nopack"])
    np.testing.assert_array_equal(out["pack"], out["pack1"])
    import oracle
    rng = np.random.default_rng(21)
    nb = rng.integers(30, 81, size=96).astype(np.int32)
    R = int(nb.sum())
    bank = {"mfccs": rng.standard_normal((R, 1000), dtype=np.float32),
            "ssms": np.abs(rng.standard_normal((R, 1225), dtype=np.float32)),
            "chromas": np.abs(rng.standard_normal((R, 480), dtype=np.float32)),
            "chroma_med": np.abs(rng.standard_normal((96, 12), dtype=np.float32)),
            "nb": nb, "off": np.concatenate([[0], np.cumsum(nb[:-1])]).astype(np.int64)}
    pairs = np.array([(i, j) for i in range(96) for j in range(96) if i != j], np.int32)
    idx = np.random.default_rng(4).choice(len(pairs), 100, replace=False)
    ref = oracle.ef_batch(bank, pairs[idx], 0.1)
    np.testing.assert_array_equal(out["pack"][idx], np.asarray(ref, np.float64))


def test_wcsm_and_neg_exp_equal_canonical_oracle():
    """acoss_wcsm (k_kmean wave-per-line canonical means + canon_expf) and acoss_neg_exp equal the
    oracle's or_ef_wcsm / canon_expf bit for bit: ties, k1 != k2, a NaN row, large k."""
    from acoss import _lib
    rng = np.random.default_rng(17)
    for M, N, k1, k2 in ((50, 60, 10, 10), (130, 77, 3, 40), (33, 500, 33, 100)):
        D = np.abs(rng.standard_normal((M, N))).astype(np.float32)
        D[3, : N // 2] = D[3, 0]
        D[: M // 2, 5] = D[0, 5]
        D[7] = np.nan
        got = _lib.wcsm(D, k1, k2, 0.5).cpu().numpy()
        ref = oracle.ef_wcsm(D, k1, k2, 0.5)
        same = (got == ref) | (np.isnan(got) & np.isnan(ref))
        assert same.all(), (M, N, k1, k2, np.argwhere(~same)[:5])
    x = np.concatenate([rng.uniform(-90, 110, 20000), rng.exponential(2.0, 20000), [0.0, -0.0, np.inf, -np.inf]])
    x = x.astype(np.float32)
    np.testing.assert_array_equal(_lib.neg_exp(x).cpu().numpy(), oracle.canon_expf(-x))


def test_earlyfusion_short_tracks_ties_equal_canonical_oracle():
    """Da-TACOS-sized tracks (14..47 beat blocks) with integer-valued block features, so the CSMs are
    full of exactly equal distances (and whole duplicate blocks: zero distances): the row-per-lane
    binarize (k_ef_binarize_lanes) must pick the lowest columns among ties as the oracle does. All four
    scores == the canonical oracle on every ordered pair, for kappa = 0.1 (nn 1..5), 0.2 (nn up to 9:
    the 4-wave kernel) and a count of 3."""
    import torch
    from acoss import _lib
    rng = np.random.default_rng(77)
    nbs = [int(v) for v in rng.integers(14, 48, size=20)]
    R = sum(nbs)
    host = {"mfccs": rng.integers(-1, 2, size=(R, 1000)).astype(np.float32),
            "ssms": rng.integers(0, 2, size=(R, 1225)).astype(np.float32),
            "chromas": rng.integers(0, 3, size=(R, 480)).astype(np.float32),
            "chroma_med": rng.integers(0, 4, size=(len(nbs), 12)).astype(np.float32),
            "nb": np.array(nbs, np.int32), "off": np.concatenate([[0], np.cumsum(nbs[:-1])]).astype(np.int64)}
    host["mfccs"][5] = host["mfccs"][9]  # duplicate blocks: zero distances
    host["chromas"][5] = host["chromas"][9]
    bank = {k: torch.as_tensor(host[k]).cuda() for k in ("mfccs", "ssms", "chromas", "chroma_med", "off", "nb")}
    bank["max_blocks"] = max(nbs)
    pairs = np.array([(i, j) for i in range(len(nbs)) for j in range(len(nbs)) if i != j], np.int32)
    for kappa in (0.1, 0.2, 3.0):
        got = _lib.earlyfusion(bank, pairs, kappa, 10).cpu().numpy()
        ref = oracle.ef_batch(host, pairs, kappa, K=10)
        bad = np.argwhere(got != ref)
        assert len(bad) == 0, (kappa, len(bad), bad[:5])
