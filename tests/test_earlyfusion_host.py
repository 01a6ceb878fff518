"""EarlyFusion's beat-synchronous block features on the host (f3, earlyfusion_traile.py:67-154,
214-247), CPU only.

The reference resizes each beat block with skimage.transform.resize(x, (frames_per_block, d),
anti_aliasing=True, mode='constant'); skimage is absent here, so acoss's resize_block restates it
with scipy.ndimage. This test pins that restatement against a second, independent restatement of
skimage's published algorithm written with plain numpy loops (Gaussian pre-filter, sigma =
max(0, (factor - 1) / 2), kernel radius int(4 sigma + 0.5), zero padding; then linear
interpolation at input coordinate (k + 0.5) * factor - 0.5 with zeros outside the block, i.e.
ndimage.zoom(grid_mode=True, mode='grid-constant')). Both are restatements: parity with skimage
itself stays unpinned. The SSM feature is pinned against the reference's get_ssm (np_oracle,
golden-pinned) taken on the upper triangle, and the block layout against the reference's loop.
"""
import numpy as np
import pytest

from oracle import np_oracle as npo


def _gauss_kernel(sigma):
    r = int(4.0 * sigma + 0.5)
    x = np.arange(-r, r + 1, dtype=np.float64)
    w = np.exp(-0.5 * x * x / (sigma * sigma))
    return w / w.sum(), r


def _resize_direct(x, n_out):
    x = np.asarray(x, np.float64)
    n_in, d = x.shape
    factor = n_in / float(n_out)
    sigma = max(0.0, (factor - 1.0) / 2.0)
    if sigma > 0:
        w, r = _gauss_kernel(sigma)
        f = np.zeros_like(x)
        for i in range(n_in):
            for t in range(-r, r + 1):
                if 0 <= i + t < n_in:
                    f[i] += w[t + r] * x[i + t]
    else:
        f = x.copy()
    out = np.zeros((n_out, d))
    for k in range(n_out):
        c = (k + 0.5) * factor - 0.5
        i0 = int(np.floor(c))
        a = c - i0
        lo = f[i0] if 0 <= i0 < n_in else 0.0
        hi = f[i0 + 1] if 0 <= i0 + 1 < n_in else 0.0
        out[k] = (1 - a) * lo + a * hi
    return out


@pytest.mark.parametrize("n_in,n_out", [(120, 50), (50, 50), (37, 50), (400, 40), (41, 40), (12, 40)])
def test_resize_block_matches_direct_restatement(n_in, n_out):
    from acoss.algorithms.earlyfusion_traile import resize_block
    rng = np.random.default_rng(n_in * 7 + n_out)
    X = rng.normal(size=(n_in + 30, 20)).astype(np.float32)
    got = resize_block(X, 10, 10 + n_in, n_out)
    np.testing.assert_allclose(got, _resize_direct(X[10:10 + n_in], n_out), rtol=1e-12, atol=1e-12)


def test_oracle_block_features_match_reference_loop():
    """np_oracle.ef_block_features (the checker of the GPU kernel acoss_ef_block_features) vs the
    reference's loop (:107-126) built from the pinned pieces: resize (restated above),
    z-normalisation, get_ssm upper triangle."""
    rng = np.random.default_rng(3)
    n = 900
    chroma = np.abs(rng.normal(size=(n, 12))).astype(np.float32)
    mfcc_htk = rng.normal(size=(20, n)).astype(np.float32)
    mfcc_htk[3, 17] = np.nan  # NaN MFCCs become 0 (:98)
    onsets = np.unique(np.clip(np.arange(0, n - 1, 43) + rng.integers(0, 3, size=len(range(0, n - 1, 43))), 0, n - 1))
    bf = npo.ef_block_features(chroma, mfcc_htk, onsets)
    mfcc = mfcc_htk.T.copy()
    mfcc[np.isnan(mfcc)] = 0
    nb = len(onsets) - 20
    assert bf["mfccs"].shape == (nb, 50 * 20) and bf["ssms"].shape == (nb, 1225) and bf["chromas"].shape == (nb, 480)
    pix = np.arange(50)
    I, J = np.meshgrid(pix, pix)
    for b in range(nb):
        x = _resize_direct(mfcc[onsets[b]:onsets[b + 19]], 50)
        x -= np.mean(x, 0)[None, :]
        xnorm = np.sqrt(np.sum(x ** 2, 1))[:, None]
        xnorm[xnorm == 0] = 1
        xn = x / xnorm
        np.testing.assert_allclose(bf["mfccs"][b], xn.flatten().astype(np.float32), rtol=2e-6, atol=1e-7)
        np.testing.assert_allclose(bf["ssms"][b], npo.get_ssm(xn)[I < J].astype(np.float32), rtol=2e-6, atol=2e-6)
        c = _resize_direct(chroma[onsets[b]:onsets[b + 20]], 40)
        np.testing.assert_allclose(bf["chromas"][b], c.flatten().astype(np.float32), rtol=2e-6, atol=1e-7)
    np.testing.assert_array_equal(bf["chroma_med"], np.median(chroma, axis=0))
    # the product's public resize_block and the oracle's are the same restatement
    from acoss.algorithms.earlyfusion_traile import resize_block
    np.testing.assert_array_equal(resize_block(mfcc, 5, 300, 50), npo.resize_block(mfcc, 5, 300, 50))


def _reference_raises(nq, nr, kappa, K):
    """Run the reference's own partition calls of one EarlyFusion pair (csm_to_binary,
    cross_recurrence.py:150-156, then getWCSM, similarity_fusion.py:47-50) on a (nq, nr) CSM."""
    D = np.arange(nq * nr, dtype=np.float32).reshape(nq, nr)
    try:
        if kappa != 0:
            np.argpartition(D, npo.nneighbs(kappa, nr), 1)
        np.partition(D, K, 1)
        np.partition(D, K, 0)
    except ValueError:
        return True
    return False


@pytest.mark.parametrize("kappa", [0.0, 0.1, 0.5, 0.95, 3.0, 12.0])
def test_ef_neighbour_error_matches_reference_partition(kappa):
    """acoss._lib.ef_neighbour_error (the host check acoss_earlyfusion's wrapper runs before the
    kernels) rejects exactly the block counts the reference's argpartition / partition reject: a
    kappa >= 1 above a track's block count, or K >= either track's block count."""
    from acoss import _lib
    for K in (1, 3, 10):
        for nq in range(1, 16):
            for nr in range(1, 16):
                err = _lib.ef_neighbour_error([nq], [nr], kappa, K)
                assert (err is not None) == _reference_raises(nq, nr, kappa, K), (nq, nr, kappa, K)
