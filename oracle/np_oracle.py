"""NumPy restatements of the acoss helpers on the hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module
(the product path is the HIP library; it never calls into oracle/). Each function cites the
reference file:line it follows. Pinned by tests/test_oracle_golden.py against the golden
vectors in tests/golden/reference_golden.npz (made by running the reference's own Python
functions, tests/golden/make_golden.py), except where a docstring says "unpinned": those
depend on librosa, which is absent from this image, and are restated from its published
algorithm (librosa 0.6.x `util.sync`, `util.normalize`, `filters.get_window`).
"""
import numpy as np
from scipy import signal


# acoss/algorithms/utils/cross_recurrence.py:10-28
def get_ssm(X):
    XSqr = np.sum(X ** 2, 1)
    DSqr = XSqr[:, None] + XSqr[None, :] - 2 * X.dot(X.T)
    DSqr[DSqr < 0] = 0
    np.fill_diagonal(DSqr, 0)
    return np.sqrt(DSqr)


# cross_recurrence.py:30-51
def get_csm(X, Y):
    C = np.sum(X ** 2, 1)[:, None] + np.sum(Y ** 2, 1)[None, :] - 2 * X.dot(Y.T)
    C[C < 0] = 0
    return np.sqrt(C)


# cross_recurrence.py:53-73
def get_csm_cosine(X, Y):
    XNorm = np.sqrt(np.sum(X ** 2, 1))
    XNorm[XNorm == 0] = 1
    YNorm = np.sqrt(np.sum(Y ** 2, 1))
    YNorm[YNorm == 0] = 1
    return 1 - (X / XNorm[:, None]).dot((Y / YNorm[:, None]).T)


# cross_recurrence.py:75-103 (np.argmax: first maximum)
def get_oti(C1, C2):
    scores = np.array([np.sum(np.roll(C1, i) * C2) for i in range(len(C1))])
    return int(np.argmax(scores))


# cross_recurrence.py:105-134
def get_csm_blocked_oti(X, Y, C1, C2, csm_fn):
    oti = get_oti(C1, C2)
    X1 = np.roll(X.reshape(X.shape[0], -1, len(C1)), oti, axis=2).reshape(X.shape[0], -1)
    return csm_fn(X1, Y)


def nneighbs(kappa, ncols):
    """csm_to_binary's neighbour count (cross_recurrence.py:150-155)."""
    return int(np.round(kappa * ncols)) if kappa < 1 else int(kappa)


# cross_recurrence.py:136-161, with ties resolved lowest column first (the reference's
# argpartition choice is unspecified; on the golden tie case it is the lowest columns)
def csm_to_binary(D, kappa):
    if kappa == 0:
        return np.ones_like(D)
    nn = nneighbs(kappa, D.shape[1])
    B = np.zeros(D.shape, np.uint8)
    cols = np.arange(D.shape[1])
    for i in range(D.shape[0]):
        B[i, np.lexsort((cols, D[i]))[:nn]] = 1
    return B


# acoss/algorithms/utils/similarity_fusion.py:38-54
def getWCSM(CSMAB, k1, k2, Mu=0.5):
    MeanDist1 = np.mean(np.partition(CSMAB, k2, 1)[:, 0:k2], 1)
    MeanDist2 = np.mean(np.partition(CSMAB, k1, 0)[0:k1, :], 0)
    Eps = (MeanDist1[:, None] + MeanDist2[None, :] + CSMAB) / 3
    return np.exp(-CSMAB ** 2 / (2 * (Mu * Eps) ** 2))


# acoss/algorithms/rqa_serra09.py:44-53 via librosa.util.sync(X, idx, aggregate=np.median)
# (librosa 0.6.1, unpinned: librosa is absent). Segments [0,40), [40,80), ..., [40k, n).
def median_downsample(chroma, factor=40):
    n = chroma.shape[0]
    bounds = list(range(0, n, factor)) + [n]
    out = np.empty((len(bounds) - 1, chroma.shape[1]), dtype=chroma.dtype)
    for s in range(len(bounds) - 1):
        out[s] = np.median(chroma[bounds[s]:bounds[s + 1]], axis=0)
    return out


# acoss/algorithms/simple_silva.py:34-43,56-66 (librosa get_window/normalize restated, unpinned)
def simple_features(chroma, win=200, skip=100, win_len_smooth=4):
    feat_orig = chroma.T
    new_feat = np.zeros((feat_orig.shape[0], int(feat_orig.shape[1] / skip)))
    for i in range(new_feat.shape[1]):
        new_feat[:, i] = np.mean(feat_orig[:, i * skip:i * skip + win], axis=1)
    w = signal.get_window("hann", win_len_smooth + 2, fftbins=False)
    w = np.atleast_2d(w / np.sum(w))
    feat = signal.convolve2d(new_feat, w, mode="same", boundary="fill")
    length = np.sqrt(np.sum(feat ** 2, axis=0))
    length[length < np.finfo(feat.dtype).tiny] = 1.0  # librosa normalize(fill=None)
    return feat / length


# acoss/algorithms/simple_silva.py:45-54
def simple_oti(seq_a, seq_b):
    pa, pb = np.sum(seq_a, 1), np.sum(seq_b, 1)
    v = np.array([np.dot(pa, np.roll(pb, i)) for i in range(12)])
    k = int(np.argsort(v, kind="stable")[-1])
    return np.roll(seq_b, k, axis=0), k


# acoss/algorithms/earlyfusion_traile.py:214-247 (resize_block, skimage.transform.resize restated:
# skimage is absent, unpinned)
def resize_block(X, i1, i2, frames_per_block):
    from scipy import ndimage
    x = np.asarray(X[i1:i2, :], dtype=np.float64)
    factor = x.shape[0] / float(frames_per_block)
    sigma = max(0.0, (factor - 1.0) / 2.0)
    if sigma > 0:
        x = ndimage.gaussian_filter(x, (sigma, 0.0), mode="constant", cval=0.0)
    ret = ndimage.zoom(x, (frames_per_block / float(x.shape[0]), 1.0), order=1, mode="grid-constant", cval=0.0,
                       grid_mode=True)
    ret[np.isinf(ret)] = 0
    ret[np.isnan(ret)] = 0
    return ret


# acoss/algorithms/earlyfusion_traile.py:100-150 (the block loops of EarlyFusion.load_features)
def ef_block_features(chroma, mfcc_htk, onsets, blocksize=20, mfccs_per_block=50, chromas_per_block=40):
    mfcc = np.array(mfcc_htk).T
    mfcc[np.isnan(mfcc)] = 0
    n_blocks = len(onsets) - blocksize
    bf = {"mfccs": np.zeros((n_blocks, mfccs_per_block * mfcc.shape[1]), dtype=np.float32)}
    pix = np.arange(mfccs_per_block)
    I, J = np.meshgrid(pix, pix)
    bf["ssms"] = np.zeros((n_blocks, int(mfccs_per_block * (mfccs_per_block - 1) / 2)), dtype=np.float32)
    for b in range(n_blocks):
        x = resize_block(mfcc, onsets[b], onsets[b + blocksize - 1], mfccs_per_block)
        x -= np.mean(x, 0)[None, :]
        xnorm = np.sqrt(np.sum(x ** 2, 1))[:, None]
        xnorm[xnorm == 0] = 1
        xn = x / xnorm
        bf["mfccs"][b, :] = xn.flatten()
        bf["ssms"][b, :] = get_ssm(xn)[I < J]
    bf["chromas"] = np.zeros((n_blocks, chromas_per_block * chroma.shape[1]), dtype=np.float32)
    bf["chroma_med"] = np.median(chroma, axis=0)
    for b in range(n_blocks):
        x = resize_block(chroma, onsets[b], onsets[b + blocksize], chromas_per_block)
        bf["chromas"][b, :] = x.flatten()
    return bf


def snf_step(mats, skip, J, V, reg_diag):
    """One cross-diffusion step of doSimilarityFusionWs for matrix `skip`
    (acoss/algorithms/utils/similarity_fusion.py:163-174): the average of the other matrices,
    then S.dot((S.dot(A.T)).T) with S the csr matrix getS builds from (J, V) (:137-142),
    then reg_diag added on the diagonal. float64 throughout, as the reference from its second
    iteration on."""
    from scipy import sparse
    n, K = J.shape
    A = np.zeros((n, n))
    for k, M in enumerate(mats):
        if k != skip:
            A += M
    A /= float(len(mats) - 1)
    S = sparse.coo_matrix((V.ravel(), (np.repeat(np.arange(n), K), J.ravel())), shape=(n, n)).tocsr()
    out = S.dot((S.dot(A.T)).T)
    if reg_diag > 0:
        out[np.arange(n), np.arange(n)] += reg_diag
    return out


def snf_fused(Ds, K=5, niters=5, reg_diag=1):
    """doSimilarityFusion (similarity_fusion.py:15-36 getW, :98-119 getP, :121-143 getS,
    :145-182 doSimilarityFusionWs, :184-192) restated around snf_step, including the reference's
    `Pts = nextPts` aliasing (from the second iteration on, matrix i sees the new k < i)."""
    Ws = []
    for D in Ds:
        DSym = 0.5 * (D + D.T)
        np.fill_diagonal(DSym, 0)
        Neighbs = np.partition(DSym, K + 1, 1)[:, 0:K + 1]
        MeanDist = np.mean(Neighbs, 1) * float(K + 1) / float(K)
        Eps = (MeanDist[:, None] + MeanDist[None, :] + DSym) / 3
        Denom = 2 * (0.5 * Eps) ** 2
        Denom[Denom == 0] = 1
        Ws.append(np.exp(-DSym ** 2 / Denom))
    Pts, JV = [], []
    for W in Ws:
        RowSum = np.sum(W, 1)
        RowSum[RowSum == 0] = 1
        Pts.append((W / RowSum[:, None]).astype(np.float64))
        J = np.argpartition(-W, K, 1)[:, 0:K]
        V = W[np.repeat(np.arange(W.shape[0]), K), J.ravel()].reshape(J.shape)
        SNorm = np.sum(V, 1)
        SNorm[SNorm == 0] = 1
        JV.append((J, (V / SNorm[:, None]).astype(np.float64)))
    L = len(Pts)
    for it in range(niters):
        nxt = list(Pts) if it == 0 else Pts
        for i in range(L):
            nxt[i] = snf_step(Pts, i, JV[i][0], JV[i][1], reg_diag)
        Pts = nxt
    return _fused_sum(Pts)


def _fused_sum(Pts):
    F = np.zeros(Pts[0].shape)
    for P in Pts:
        F += P
    return F / len(Pts)
