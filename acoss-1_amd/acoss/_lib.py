"""ctypes binding of libacoss_hip.so (the C-ABI declared in include/acoss_hip.h).

This is the only door from Python into the HIP kernels. There is no CPU fallback: if the
library or a GPU is missing, every entry point raises ``AcossHipError``.

Device memory is owned by torch tensors; pointers go through ``Tensor.data_ptr()`` and
calls are ordered on the current torch stream.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ACOSS_HIP_LIB", os.path.join(_HERE, "lib", "libacoss_hip.so"))

ACOSS_OK = 0
_ERRNAMES = {-1: "ACOSS_E_ARG", -2: "ACOSS_E_SHAPE", -3: "ACOSS_E_HIP", -4: "ACOSS_E_NONBINARY"}


class AcossHipError(RuntimeError):
    """Raised on any failure of the HIP engine (missing library, no GPU, kernel error)."""


class CrpParams(ctypes.Structure):
    """acoss_crp_params — essentia ChromaCrossSimilarity/CoverSongSimilarity parameters
    (acoss/algorithms/rqa_serra09.py:31-32,60-64)."""
    _fields_ = [("m", ctypes.c_int32), ("tau", ctypes.c_int32), ("kappa", ctypes.c_float),
                ("oti", ctypes.c_int32), ("gamma_open", ctypes.c_float), ("gamma_ext", ctypes.c_float)]


_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f32 = ctypes.c_float

# name -> argtypes; every function returns int
SIGNATURES = {
    "acoss_crp_align": [_vp, _vp, _vp, _i32, _i32, _vp, _i64, ctypes.POINTER(CrpParams), _vp, _vp, _vp, _vp],
    "acoss_crp_pair": [_vp, _i32, _vp, _i32, ctypes.POINTER(CrpParams), _vp, _vp, _vp, _vp, _vp, _vp],
    "acoss_align_crp": [_vp, _i32, _i32, _i32, _f32, _f32, _vp, _vp],
    "acoss_sw_constrained": [_vp, _vp, _vp, _vp, _i32, _i32, _i32, _vp, _vp],
    "acoss_csm": [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp],
    "acoss_get_oti": [_vp, _vp, _i32, _vp, _vp],
    "acoss_binarize_rows": [_vp, _i32, _i32, _i32, _vp, _vp],
    "acoss_wcsm": [_vp, _i32, _i32, _i32, _i32, _f32, _vp, _vp],
    "acoss_simple_mp": [_vp, _vp, _vp, _i32, _i32, _vp, _i64, _i32, _vp, _vp, _vp],
    "acoss_release_workspace": [],
    "acoss_profile_enable": [ctypes.c_int],
    "acoss_profile_read": [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64), ctypes.c_int],
}

_lib = None


def load_library(path=None):
    """Load (once) and return the ctypes handle. Raises AcossHipError if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise AcossHipError(
            "libacoss_hip.so not found at %s: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(or `make -C acoss-1_amd/csrc`). There is no CPU fallback." % p)
    lib = ctypes.CDLL(p)
    for name, argt in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argt
        fn.restype = ctypes.c_int
    lib.acoss_last_error.restype = ctypes.c_char_p
    lib.acoss_last_error.argtypes = []
    lib.acoss_version.restype = ctypes.c_char_p
    lib.acoss_version.argtypes = []
    lib.acoss_profile_phase_name.restype = ctypes.c_char_p
    lib.acoss_profile_phase_name.argtypes = [ctypes.c_int]
    if path is None:
        _lib = lib
    return lib


def _check(rc, what):
    if rc != ACOSS_OK:
        msg = load_library().acoss_last_error().decode(errors="replace")
        raise AcossHipError("%s failed (%s): %s" % (what, _ERRNAMES.get(rc, rc), msg))


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise AcossHipError("no HIP GPU visible to torch: the acoss HIP engine has no CPU fallback")
    return torch


def _stream():
    torch = _torch()
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _dev(x, dtype):
    """numpy/torch -> contiguous device tensor of `dtype`."""
    torch = _torch()
    if isinstance(x, torch.Tensor):
        return x.to(device="cuda", dtype=dtype).contiguous()
    return torch.as_tensor(np.ascontiguousarray(x)).to(device="cuda", dtype=dtype).contiguous()


def crp_params(m=9, tau=1, kappa=0.095, oti=True, gamma_open=0.5, gamma_ext=0.5):
    return CrpParams(int(m), int(tau), float(kappa), int(bool(oti)), float(gamma_open), float(gamma_ext))


# ----------------------------------------------------------------------------------------
# Thin wrappers: inputs/outputs are torch CUDA tensors.
# ----------------------------------------------------------------------------------------
def crp_align(feats, track_off, track_len, max_len, pairs, params, qmax=True, dmax=False, oti=False):
    """Batched Serra09/Chen path. feats (sum_n, 12) f32, track_off (T,) i64, track_len (T,) i32,
    pairs (P, 2) i32 (query, reference) -> dict of device tensors."""
    torch = _torch()
    lib = load_library()
    feats = _dev(feats, torch.float32)
    track_off = _dev(track_off, torch.int64)
    track_len = _dev(track_len, torch.int32)
    pairs = _dev(pairs, torch.int32)
    P = pairs.shape[0]
    out = {}
    q = torch.empty(P, dtype=torch.float32, device="cuda") if qmax else None
    d = torch.empty(P, dtype=torch.float32, device="cuda") if dmax else None
    o = torch.empty(P, dtype=torch.int32, device="cuda") if oti else None
    rc = lib.acoss_crp_align(_ptr(feats), _ptr(track_off), _ptr(track_len), int(track_len.shape[0]), int(max_len),
                             _ptr(pairs), int(P), ctypes.byref(params), _ptr(q), _ptr(d), _ptr(o), _stream())
    _check(rc, "acoss_crp_align")
    if qmax:
        out["qmax"] = q
    if dmax:
        out["dmax"] = d
    if oti:
        out["oti"] = o
    return out


def crp_pair(X, Y, params, dist=True):
    """Single pair with intermediates: dist, thr_row, thr_col, crp (uint8), oti."""
    torch = _torch()
    lib = load_library()
    X = _dev(X, torch.float32)
    Y = _dev(Y, torch.float32)
    M, N = X.shape[0], Y.shape[0]
    m, tau = params.m, params.tau
    Mp = max(0, -(-(M - m * tau) // tau)) if M > m * tau else 0
    Np = max(0, -(-(N - m * tau) // tau)) if N > m * tau else 0
    D = torch.empty((Mp, Np), dtype=torch.float32, device="cuda") if dist else None
    tr = torch.empty(Mp, dtype=torch.float32, device="cuda")
    tc = torch.empty(Np, dtype=torch.float32, device="cuda")
    C = torch.empty((Mp, Np), dtype=torch.uint8, device="cuda")
    o = torch.empty(1, dtype=torch.int32, device="cuda")
    rc = lib.acoss_crp_pair(_ptr(X), M, _ptr(Y), N, ctypes.byref(params), _ptr(D), _ptr(tr), _ptr(tc), _ptr(C),
                            _ptr(o), _stream())
    _check(rc, "acoss_crp_pair")
    return {"dist": D, "thr_row": tr, "thr_col": tc, "crp": C, "oti": o}


def align_crp(C, align=0, gamma_open=0.5, gamma_ext=0.5):
    """essentia CoverSongSimilarity(serra09|chen17, 'symmetric') on a binary (M, N) matrix."""
    torch = _torch()
    lib = load_library()
    C = _dev(C, torch.uint8)
    out = torch.empty(1, dtype=torch.float32, device="cuda")
    rc = lib.acoss_align_crp(_ptr(C), int(C.shape[0]), int(C.shape[1]), int(align), float(gamma_open),
                             float(gamma_ext), _ptr(out), _stream())
    _check(rc, "acoss_align_crp")
    return out


def profile_enable(on=True):
    load_library().acoss_profile_enable(1 if on else 0)


def profile_read():
    """{phase name: (total_ms, launches)} for the phases recorded since profile_enable(True)."""
    lib = load_library()
    n = 32
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_int64 * n)()
    k = lib.acoss_profile_read(ms, cnt, n)
    if k < 0:
        _check(k, "acoss_profile_read")
    return {lib.acoss_profile_phase_name(i).decode(): (ms[i], int(cnt[i])) for i in range(k) if cnt[i] > 0}
