"""Edge cases of the batched entry points on the GPU: empty pair lists, one-track and two-track
corpora, a 1 x 1 score matrix, the evaluation of a corpus of singletons. Each must return the
reference's answer (empty arrays, zero rows, nan/inf where the reference has them) without a
kernel launch on empty grids."""
import numpy as np
import pytest

import oracle
from acoss import _lib, evaluation, synthetic

pytestmark = pytest.mark.gpu


def _tracks(lengths, seed=5):
    rng = np.random.Generator(np.random.PCG64(seed))
    return [synthetic.render(rng, synthetic.base_sequence(rng, n)) for n in lengths]


def test_crp_align_no_pairs():
    feats, off, lens = synthetic.pack(_tracks([200, 300]))
    got = _lib.crp_align(feats, off, lens, int(lens.max()), np.zeros((0, 2), np.int32), _lib.crp_params(),
                         qmax=True, dmax=True, oti=True)
    assert got["qmax"].numel() == 0 and got["dmax"].numel() == 0 and got["oti"].numel() == 0


def test_crp_align_one_pair_and_self_pair():
    """A single pair (one-wave launches everywhere) and a track against itself, both == oracle."""
    feats, off, lens = synthetic.pack(_tracks([230, 260]))
    pairs = np.array([[0, 1], [1, 1]], np.int32)
    q, d, k = oracle.crp_batch(feats, off, lens, pairs)
    for sel in ([0], [1], [0, 1]):
        got = _lib.crp_align(feats, off, lens, int(lens.max()), pairs[sel], _lib.crp_params(), qmax=True, dmax=True,
                             oti=True)
        np.testing.assert_array_equal(got["qmax"].cpu().numpy(), q[sel])
        np.testing.assert_array_equal(got["dmax"].cpu().numpy(), d[sel])
        np.testing.assert_array_equal(got["oti"].cpu().numpy(), k[sel])


def test_simple_no_pairs():
    import torch
    F = np.random.default_rng(1).random((12, 50))
    score, oti = _lib.simple_mp_packed(torch.as_tensor(F.ravel()).cuda(), [0], [50], np.zeros((0, 2), np.int32))
    assert score.numel() == 0 and oti.numel() == 0


def test_earlyfusion_no_pairs():
    import torch
    NB = 30
    rng = np.random.default_rng(2)
    bank = {"mfccs": torch.as_tensor(rng.standard_normal((2 * NB, 1000), dtype=np.float32)).cuda(),
            "ssms": torch.as_tensor(np.abs(rng.standard_normal((2 * NB, 1225), dtype=np.float32))).cuda(),
            "chromas": torch.as_tensor(np.abs(rng.standard_normal((2 * NB, 480), dtype=np.float32))).cuda(),
            "chroma_med": torch.as_tensor(np.abs(rng.standard_normal((2, 12), dtype=np.float32))).cuda(),
            "off": torch.as_tensor(np.array([0, NB], np.int64)).cuda(),
            "nb": torch.as_tensor(np.array([NB, NB], np.int32)).cuda(), "max_blocks": NB}
    assert _lib.earlyfusion(bank, np.zeros((0, 2), np.int32)).shape == (0, 4)
    one = _lib.earlyfusion(bank, np.array([[0, 1]], np.int32)).cpu().numpy()
    assert one.shape == (1, 4) and np.isfinite(one).all()


def test_earlyfusion_rejects_neighbours_beyond_blocks():
    """kappa >= 1 with int(kappa) >= a track's block count, or K >= a block count: the reference's
    argpartition / partition raise ValueError (cross_recurrence.py:156, similarity_fusion.py:47);
    so does the wrapper, before any kernel runs. A valid kappa >= 1 still scores."""
    import torch
    rng = np.random.default_rng(4)
    nbs = [30, 12]
    T = sum(nbs)
    bank = {"mfccs": torch.as_tensor(rng.standard_normal((T, 1000), dtype=np.float32)).cuda(),
            "ssms": torch.as_tensor(np.abs(rng.standard_normal((T, 1225), dtype=np.float32))).cuda(),
            "chromas": torch.as_tensor(np.abs(rng.standard_normal((T, 480), dtype=np.float32))).cuda(),
            "chroma_med": torch.as_tensor(np.abs(rng.standard_normal((2, 12), dtype=np.float32))).cuda(),
            "off": torch.as_tensor(np.array([0, nbs[0]], np.int64)).cuda(),
            "nb": torch.as_tensor(np.array(nbs, np.int32)).cuda(), "max_blocks": max(nbs)}
    with pytest.raises(ValueError, match="out of bounds"):
        _lib.earlyfusion(bank, np.array([[0, 1]], np.int32), kappa=12.0, K=5)   # 12 >= 12 columns
    with pytest.raises(ValueError, match="out of bounds"):
        _lib.earlyfusion(bank, np.array([[1, 0]], np.int32), kappa=0.1, K=12)   # K >= 12 rows
    ok = _lib.earlyfusion(bank, np.array([[0, 1], [1, 0]], np.int32), kappa=11.0, K=5).cpu().numpy()
    assert np.isfinite(ok).all()


def test_ds_finish_one_by_one():
    import torch
    D = torch.full((1, 1), 3.0, dtype=torch.float32, device="cuda")
    _lib.ds_finish(D, symmetric=True)
    assert float(D[0, 0]) == 6.0
    D = torch.full((1, 1), 3.0, dtype=torch.float32, device="cuda")
    _lib.ds_finish(D, norm=np.array([2.0]), symmetric=False, mode="serra09")
    assert float(D[0, 0]) == np.float32(3.0 / 2.0)


def test_eval_singletons_and_pairs_only():
    """A corpus of singletons has no queries (the reference's MAP of an empty mean is nan); one
    two-song clique among singletons gives that clique's two queries only."""
    import warnings
    import torch
    rng = np.random.default_rng(3)
    D = rng.random((6, 6)).astype(np.float32)
    Dd = torch.as_tensor(D).cuda()
    labels = np.arange(6)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        host = evaluation.eval_statistics(D, labels)
        dev = evaluation.eval_statistics_device(Dd, labels)
    for h, g in zip(host[:4], dev[:4]):
        assert (np.isnan(h) and np.isnan(g)) or h == g
    labels = np.array([0, 0, 1, 2, 3, 4])
    host = evaluation.eval_statistics(D, labels)
    dev = evaluation.eval_statistics_device(Dd, labels)
    np.testing.assert_array_equal(np.asarray(host[:4], np.float64), np.asarray(dev[:4], np.float64))
    np.testing.assert_array_equal(host[4], dev[4])
