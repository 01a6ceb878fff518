"""Whole-corpus parity of the Serra09 path and the device finish/evaluation (GPU).

* Every one of the 13,366 unordered pairs of a covers80-shaped corpus through the HIP path and
  through the oracle: Qmax bit-exact, the finished matrices (Ds += Ds.T, then / sqrt(n_j),
  rqa_serra09.py:71-83) bit-exact, and MR/MRR/MDR/MAP/Top-k identical
  (algorithm_template.py:206-291). The corpus is the discriminative one
  (synthetic.make_hard_corpus), whose MAP sits well below 1, so a differing score matrix can
  move the statistics.
* The batching branches a Da-TACOS run takes (several DP batches, several key-plane
  sub-batches, three streams: crp.hip acoss_crp_align) on a ragged corpus, against the oracle
  with ==.
* acoss_ds_finish and acoss_eval_ranks against numpy with ties, inf and NaN.
"""
import os

import numpy as np
import pytest

import oracle
from acoss import _lib, evaluation, synthetic

pytestmark = pytest.mark.gpu


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def _all_pairs(T):
    return np.array([(i, j) for i in range(T) for j in range(i + 1, T)], np.int32)


def _finish_host(q, pairs, lens):
    T = len(lens)
    D = np.zeros((T, T), np.float32)
    D[pairs[:, 0], pairs[:, 1]] = q
    D = D + D.T
    return (D / np.sqrt(lens.astype(np.float64))[None, :]).astype(np.float32)


def test_full_corpus_qmax_and_map_parity_500():
    import torch
    from acoss.engine import ChromaBank
    tracks, labels = synthetic.make_hard_corpus("covers80", frames=500)
    T = len(tracks)
    assert T == 164
    lens = np.array([len(t) for t in tracks], np.int32)
    pairs = _all_pairs(T)
    assert len(pairs) == 13366
    bank = ChromaBank(tracks)
    gq = bank.crp_align(pairs, qmax=True)["qmax"]
    feats, off, ln = synthetic.pack(tracks)
    oq, _, _ = oracle.crp_batch(feats, off, ln, pairs, dmax=False, nthreads=_threads())
    np.testing.assert_array_equal(gq.cpu().numpy(), oq)
    # device finish (scatter, symmetrise, normalise) == the reference's host arithmetic
    Dg = torch.zeros((T, T), dtype=torch.float32, device="cuda")
    p = torch.as_tensor(pairs.astype(np.int64)).cuda()
    Dg[p[:, 0], p[:, 1]] = gq
    _lib.ds_finish(Dg, symmetric=True)
    _lib.ds_finish(Dg, np.sqrt(lens.astype(np.float64)), symmetric=False, mode="serra09")
    Do = _finish_host(oq, pairs, lens)
    np.testing.assert_array_equal(Dg.cpu().numpy(), Do)
    sg = evaluation.eval_statistics_device(Dg, labels=labels)
    so = evaluation.eval_statistics(Do, labels)
    for a, b in zip(sg[:4], so[:4]):
        assert a == b
    np.testing.assert_array_equal(sg[4], so[4])
    MAP = so[3]
    assert 0.3 < MAP < 0.9, MAP  # discriminative: a changed matrix can move it


@pytest.mark.parametrize("env", [
    {"ACOSS_BATCH_PAIRS": "7"},                                   # many DP batches
    {"ACOSS_KEY_BYTES": str(20 << 20)},                           # ~2 pairs per key-plane sub-batch
    {"ACOSS_SPLIT_STREAMS": "3", "ACOSS_KEY_BYTES": str(40 << 20)},
    {"ACOSS_BATCH_PAIRS": "5", "ACOSS_SPLIT_STREAMS": "1", "ACOSS_KEY_BYTES": "1"},  # 1 pair per sub-batch
    {"ACOSS_SPLIT_STREAMS": "2", "ACOSS_KEY_BYTES": "1"},         # 1-pair sub-batches on two streams
    {"ACOSS_WS_BYTES": str(48 << 20)},                            # DP batches from a small workspace budget
])
def test_batching_branches_ragged(monkeypatch, env):
    from acoss.engine import ChromaBank
    rng = np.random.default_rng(21)
    lens = rng.integers(120, 1400, size=22)
    tracks = [synthetic.render(rng, synthetic.base_sequence(rng, int(n))) for n in lens]
    tracks[3] = synthetic.render(rng, synthetic.cover_of(rng, tracks[2], 900))
    pairs = _all_pairs(len(tracks))
    feats, off, ln = synthetic.pack(tracks)
    oq, od, ok = oracle.crp_batch(feats, off, ln, pairs, dmax=True, nthreads=_threads())
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    out = ChromaBank(tracks).crp_align(pairs, qmax=True, dmax=True, want_oti=True)
    np.testing.assert_array_equal(out["oti"].cpu().numpy(), ok)
    np.testing.assert_array_equal(out["qmax"].cpu().numpy(), oq)
    np.testing.assert_array_equal(out["dmax"].cpu().numpy(), od)


@pytest.mark.parametrize("n", [1, 5, 63, 64, 65, 200])
def test_ds_finish_matches_numpy(n):
    import torch
    rng = np.random.default_rng(n)
    D = (rng.random((n, n)) * 40).astype(np.float32)
    D[np.tril_indices(n)] = 0.0
    if n > 4:
        D[0, 3] = 0.0  # a zero score: Chen's quotient is inf, as numpy's
    norm = np.sqrt(rng.integers(20, 3000, size=n).astype(np.float64))
    sym = D + D.T
    dt = torch.as_tensor(D).cuda()
    out = torch.empty_like(dt)
    _lib.ds_finish(dt, symmetric=True, out=out)
    np.testing.assert_array_equal(out.cpu().numpy(), sym)
    np.testing.assert_array_equal(dt.cpu().numpy(), D)  # out-of-place leaves D alone
    _lib.ds_finish(dt, symmetric=True)                  # in place
    np.testing.assert_array_equal(dt.cpu().numpy(), sym)
    a = dt.clone()
    _lib.ds_finish(a, norm, symmetric=False, mode="serra09")
    np.testing.assert_array_equal(a.cpu().numpy(), (sym / norm[None, :]).astype(np.float32))
    b = dt.clone()
    with np.errstate(divide="ignore"):
        ref = (norm[None, :] / sym).astype(np.float32)
    _lib.ds_finish(b, norm, symmetric=False, mode="chen")
    np.testing.assert_array_equal(b.cpu().numpy(), ref)
    # a padded row stride
    big = torch.zeros((n, n + 7), dtype=torch.float32, device="cuda")
    big[:, :n] = torch.as_tensor(D).cuda()
    view = big[:, :n]
    _lib.ds_finish(view, norm, symmetric=True, mode="serra09")
    np.testing.assert_array_equal(view.cpu().numpy(), (sym / norm[None, :]).astype(np.float32))
    assert float(big[:, n:].abs().sum()) == 0.0


def test_eval_ranks_ties_inf_nan():
    """Device ranks == the host's stable argsort ranks, with tied, infinite and NaN scores."""
    import torch
    rng = np.random.default_rng(5)
    labels = np.repeat(np.arange(30), rng.integers(1, 6, size=30))
    N = len(labels)
    D = rng.integers(0, 6, size=(N, N)).astype(np.float32)  # many exact ties
    D[rng.random((N, N)) < 0.02] = np.inf
    D[rng.random((N, N)) < 0.02] = -np.inf
    D[rng.random((N, N)) < 0.02] = np.nan
    so = evaluation.eval_statistics(D, labels)
    sg = evaluation.eval_statistics_device(torch.as_tensor(D).cuda(), labels=labels)
    for a, b in zip(sg[:4], so[:4]):
        assert (a == b) or (np.isnan(a) and np.isnan(b)), (a, b)
    np.testing.assert_array_equal(sg[4], so[4])
    # explicit cliques in dict order (CoverAlgorithm.getEvalStatistics)
    cliques = [sorted(np.flatnonzero(labels == c).tolist()) for c in np.unique(labels)[::-1]]
    so = evaluation.eval_statistics_cliques(D, cliques)
    sg = evaluation.eval_statistics_device(torch.as_tensor(D).cuda(), cliques=cliques)
    for a, b in zip(sg[:4], so[:4]):
        assert (a == b) or (np.isnan(a) and np.isnan(b)), (a, b)


