"""Cross-recurrence helpers (acoss/algorithms/utils/cross_recurrence.py) on the HIP engine.

Same names, arguments and return types as the reference (numpy in, numpy out); the work runs
in misc.hip through the C-ABI (include/acoss_hip.h). There is no CPU fallback.
"""
import numpy as np

from ... import _lib

__all__ = ["get_ssm", "get_csm", "get_csm_euclidean", "get_csm_cosine", "get_oti", "get_csm_blocked_oti",
           "csm_to_binary", "nneighbs"]


def _host(t):
    return t.detach().cpu().numpy()


def get_ssm(X):
    """Euclidean self-similarity matrix, zero diagonal (cross_recurrence.py:10-28)."""
    return _host(_lib.csm(np.asarray(X, np.float32), kind="ssm"))


def get_csm(X, Y):
    """Euclidean cross-similarity matrix (cross_recurrence.py:30-48)."""
    return _host(_lib.csm(np.asarray(X, np.float32), np.asarray(Y, np.float32), kind="euclidean"))


get_csm_euclidean = get_csm


def get_csm_cosine(X, Y):
    """1 - normalised dot products; zero rows count as norm 1 (cross_recurrence.py:53-73)."""
    return _host(_lib.csm(np.asarray(X, np.float32), np.asarray(Y, np.float32), kind="cosine"))


def get_oti(C1, C2, do_plot=False):
    """argmax_i sum(roll(C1, i) * C2), first maximum (cross_recurrence.py:75-103)."""
    return int(_host(_lib.get_oti(np.asarray(C1, np.float32), np.asarray(C2, np.float32)))[0])


def get_csm_blocked_oti(X, Y, C1, C2, csm_fn):
    """Roll every 12-bin block of X by get_oti(C1, C2), then csm_fn(X1, Y)
    (cross_recurrence.py:105-134). get_csm / get_csm_cosine fuse the roll into the GEMM."""
    oti = get_oti(C1, C2)
    kinds = {get_csm: "euclidean", get_csm_cosine: "cosine"}
    if csm_fn in kinds:
        return _host(_lib.csm(np.asarray(X, np.float32), np.asarray(Y, np.float32), kind=kinds[csm_fn],
                              oti_shift=oti))
    nb = len(C1)
    X1 = np.roll(np.reshape(X, (X.shape[0], -1, nb)), oti, axis=2).reshape(X.shape[0], -1)
    return csm_fn(X1, Y)


def nneighbs(kappa, ncols):
    """Neighbour count of csm_to_binary (cross_recurrence.py:150-155)."""
    return int(np.round(kappa * ncols)) if kappa < 1 else int(kappa)


def csm_to_binary(D, kappa):
    """Row-wise kappa-NN binarisation (cross_recurrence.py:136-161): kappa == 0 -> all ones
    (a float array, as in the reference); otherwise the round(kappa * ncols) (or kappa) smallest
    entries of each row -> 1 in a uint8 matrix. Ties: lowest column first (the reference's
    argpartition leaves the choice unspecified)."""
    D = np.asarray(D)
    if kappa == 0:
        return np.ones_like(D)
    nn = nneighbs(kappa, D.shape[1])
    if nn >= D.shape[1]:
        raise ValueError("kth(=%d) out of bounds (%d)" % (nn, D.shape[1]))  # np.argpartition's error
    return _host(_lib.binarize_rows(np.asarray(D, np.float32), nn))
