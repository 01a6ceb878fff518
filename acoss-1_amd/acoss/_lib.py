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


class NpzMember(ctypes.Structure):
    """acoss_npz_member — one array of an .npz feature file (include/acoss_hip.h)."""
    _fields_ = [("file", ctypes.c_int32), ("method", ctypes.c_int32), ("ndim", ctypes.c_int32),
                ("fortran", ctypes.c_int32), ("shape", ctypes.c_int64 * 8), ("nbytes", ctypes.c_int64),
                ("member_off", ctypes.c_int64), ("comp_size", ctypes.c_int64), ("npy_size", ctypes.c_int64),
                ("data_skip", ctypes.c_int64), ("name", ctypes.c_char * 128), ("descr", ctypes.c_char * 32)]


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
    "acoss_neg_exp": [_vp, _i64, _vp, _vp],
    "acoss_npz_index": [ctypes.POINTER(ctypes.c_char_p), _i32, ctypes.c_char_p, _i32, ctypes.POINTER(NpzMember), _i64,
                        ctypes.POINTER(ctypes.c_int64)],
    "acoss_npz_read": [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(NpzMember), _i64, ctypes.POINTER(_vp), _i32],
    "acoss_snf_step": [_vp, _i32, _i32, _i32, _vp, _vp, _i32, ctypes.c_double, _vp, _i32, _vp],
    "acoss_snf_diffuse_rows": [_vp, _i32, _i32, _i32, _i32, _vp, _vp, _i32, _vp, _i32, _vp],
    "acoss_snf_left_rows": [_vp, _i32, _i32, _i32, _vp, _vp, _i32, ctypes.c_double, _vp, _i32, _vp],
    "acoss_simple_mp": [_vp, _vp, _vp, _i32, _i32, _vp, _i64, _i32, _i32, _vp, _vp, _vp],
    "acoss_median_downsample": [_vp, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp],
    "acoss_simple_features": [_vp, _vp, _vp, _i32, _i32, _i32, _vp, _i32, _vp, _vp, _i64, _vp],
    "acoss_earlyfusion": [_vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _i64, ctypes.c_double,
                          _i32, _f32, _vp, _vp],
    "acoss_ef_block_features": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32, _i32, _i32, _vp, _vp, _vp,
                                _vp, _vp],
    "acoss_ds_finish": [_vp, _i32, _i64, _vp, _i32, _i32, _vp, _vp],
    "acoss_eval_ranks": [_vp, _i32, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _vp],
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
    # torch bundles its own libamdhip64.so.7 (same soname as /opt/rocm's): load it first so
    # this library binds to the runtime torch's allocator and streams live in
    import torch  # noqa: F401
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


_BOUND = [False]


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise AcossHipError("no HIP GPU visible to torch: the acoss HIP engine has no CPU fallback")
    if not _BOUND[0]:  # one process per GPU under RCCL: bind before the first "cuda" allocation
        from .distributed import bind_local_device
        _BOUND[0] = bind_local_device() is not None
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


def _check_pairs(pairs, n_tracks):
    """Host-side bounds check of (P, 2) track indices before a kernel dereferences them."""
    if pairs.numel() and (int(pairs.min()) < 0 or int(pairs.max()) >= n_tracks):
        raise ValueError("pair indices must lie in [0, %d)" % n_tracks)


def _pairs_dev(pairs, n_tracks):
    """(P, 2) int32 device pairs, bounds-checked. Host (numpy / list) pairs are checked on the
    host and uploaded from pinned memory without a stream synchronisation, so a caller feeding
    chunks keeps the GPU busy while it forms the next one; device tensors are checked on the
    device (two synchronising reductions). Returns (device tensor, host array or None)."""
    torch = _torch()
    if isinstance(pairs, torch.Tensor):
        d = pairs.to(device="cuda", dtype=torch.int32).reshape(-1, 2).contiguous()
        _check_pairs(d, n_tracks)
        return d, None
    h = np.ascontiguousarray(np.asarray(pairs).reshape(-1, 2), dtype=np.int32)
    if len(h) and (int(h.min()) < 0 or int(h.max()) >= n_tracks):
        raise ValueError("pair indices must lie in [0, %d)" % n_tracks)
    if len(h) == 0:
        return torch.empty((0, 2), dtype=torch.int32, device="cuda"), h
    return torch.from_numpy(h).pin_memory().to("cuda", non_blocking=True), h


def check_knn(J, n):
    """Public form of the kNN index check (see snf_step(validated=True))."""
    _check_knn(J, n)


def _check_knn(J, n):
    """Host-side check of kNN column indices (n, K) before a kernel gathers the rows they name:
    every entry in [0, n), no repeated column within a row (scipy's coo -> csr would merge a
    repeat into one term, so the product would differ from the reference)."""
    if J.numel() == 0:
        return
    if int(J.min()) < 0 or int(J.max()) >= n:
        raise ValueError("kNN column indices must lie in [0, %d)" % n)
    if J.shape[1] > 1:
        Js = J.sort(dim=1).values
        if bool((Js[:, 1:] == Js[:, :-1]).any()):
            raise ValueError("kNN column indices repeat within a row")


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
    pairs, _ = _pairs_dev(pairs, int(track_len.shape[0]))
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


def _pack_mats(mats, dtype):
    """list of 2-D arrays -> (flat device buffer, offsets i64, rows i32, cols i32, max_rows, max_cols)."""
    torch = _torch()
    shapes = [tuple(int(v) for v in m.shape) for m in mats]
    sizes = [r * c for r, c in shapes]
    off = np.zeros(len(mats), dtype=np.int64)
    if len(mats) > 1:
        off[1:] = np.cumsum(sizes[:-1])
    flat = torch.empty(max(1, int(sum(sizes))), dtype=dtype, device="cuda")
    for m, o, n in zip(mats, off, sizes):
        if n:
            flat[int(o):int(o) + n] = _dev(m, dtype).reshape(-1)
    rows = np.array([r for r, _ in shapes], dtype=np.int32)
    cols = np.array([c for _, c in shapes], dtype=np.int32)
    return (flat, _dev(off, torch.int64), _dev(rows, torch.int32), _dev(cols, torch.int32),
            int(rows.max(initial=0)), int(cols.max(initial=0)))


def _as_binary_u8(m):
    """Binary matrix -> uint8, raising like `match` (alignment_tools.py:17-23) on other values."""
    torch = _torch()
    t = m if isinstance(m, torch.Tensor) else torch.as_tensor(np.asarray(m))
    if t.dtype not in (torch.uint8, torch.bool):
        t = t.to("cuda")
        if bool(((t != 0) & (t != 1)).any()):
            raise IOError("Non-binary elements found in input")
    return t.to(device="cuda", dtype=torch.uint8)


def sw_constrained(mats):
    """smith_waterman_constrained (alignment_tools.py:27-46) of a list of binary matrices -> (n,) f64."""
    torch = _torch()
    lib = load_library()
    mats = [_as_binary_u8(m) for m in mats]
    out = torch.empty(len(mats), dtype=torch.float64, device="cuda")
    if not mats:
        return out
    flat, off, rows, cols, mr, mc = _pack_mats(mats, torch.uint8)
    rc = lib.acoss_sw_constrained(_ptr(flat), _ptr(off), _ptr(rows), _ptr(cols), len(mats), mr, mc, _ptr(out),
                                  _stream())
    if rc == -4:
        raise IOError("Non-binary elements found in input")
    _check(rc, "acoss_sw_constrained")
    return out


CSM_KINDS = {"euclidean": 0, "euclid": 0, "cosine": 1, "ssm": 2}


def csm(X, Y=None, kind="euclidean", oti_shift=0):
    """get_csm / get_csm_cosine / get_ssm (cross_recurrence.py:10-73); oti_shift > 0 rolls each
    12-bin block of X first (get_csm_blocked_oti, :105-134). float32 (M, N) device tensor."""
    torch = _torch()
    lib = load_library()
    k = CSM_KINDS[kind]
    X = _dev(X, torch.float32)
    if X.dim() != 2:
        raise ValueError("X must be 2-D")
    if k == 2:
        Yt, N = None, X.shape[0]
    else:
        Yt = _dev(Y, torch.float32)
        if Yt.dim() != 2 or Yt.shape[1] != X.shape[1]:
            raise ValueError("X and Y need the same feature dimension")
        N = Yt.shape[0]
    out = torch.empty((X.shape[0], N), dtype=torch.float32, device="cuda")
    rc = lib.acoss_csm(_ptr(X), int(X.shape[0]), _ptr(Yt), int(N), int(X.shape[1]), k, int(oti_shift), _ptr(out),
                       _stream())
    _check(rc, "acoss_csm")
    return out


def get_oti(C1, C2):
    """get_oti (cross_recurrence.py:75-103) for (n, 12) batches (or single (12,) vectors)."""
    torch = _torch()
    lib = load_library()
    a = _dev(C1, torch.float32).reshape(-1, 12)
    b = _dev(C2, torch.float32).reshape(-1, 12)
    out = torch.empty(a.shape[0], dtype=torch.int32, device="cuda")
    rc = lib.acoss_get_oti(_ptr(a), _ptr(b), int(a.shape[0]), _ptr(out), _stream())
    _check(rc, "acoss_get_oti")
    return out


def binarize_rows(D, nneighbs):
    """The nneighbs smallest of every row -> 1 (csm_to_binary, cross_recurrence.py:136-161)."""
    torch = _torch()
    lib = load_library()
    D = _dev(D, torch.float32)
    out = torch.empty(D.shape, dtype=torch.uint8, device="cuda")
    rc = lib.acoss_binarize_rows(_ptr(D), int(D.shape[0]), int(D.shape[1]), int(nneighbs), _ptr(out), _stream())
    _check(rc, "acoss_binarize_rows")
    return out


def wcsm(CSM, k1, k2, mu=0.5):
    """getWCSM (similarity_fusion.py:38-54)."""
    torch = _torch()
    lib = load_library()
    C = _dev(CSM, torch.float32)
    out = torch.empty(C.shape, dtype=torch.float32, device="cuda")
    rc = lib.acoss_wcsm(_ptr(C), int(C.shape[0]), int(C.shape[1]), int(k1), int(k2), float(mu), _ptr(out), _stream())
    _check(rc, "acoss_wcsm")
    return out


def npz_read_many(paths, keys=None, n_threads=0):
    """The arrays of many .npz files, read on native threads in two C calls (acoss_npz_index,
    acoss_npz_read; host only, no GPU, the GIL released inside both): a list (one per path, in
    order) of {member name: ndarray}, names as stored ('madmom_features/onsets'). keys: read only
    members whose top-level name is in keys (None: all). Raises IOError naming the file on an
    unreadable or unsupported file (object arrays are refused, as np.load(allow_pickle=False))."""
    lib = load_library()
    n = len(paths)
    if n == 0:
        return []
    cpaths = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
    ckeys = None if keys is None else "\n".join(keys).encode()
    cap = max(16, n * (4 if keys is not None else 8))
    while True:
        buf = (NpzMember * cap)()
        got = ctypes.c_int64(0)
        rc = lib.acoss_npz_index(cpaths, n, ckeys, int(n_threads), buf, cap, ctypes.byref(got))
        if rc == ACOSS_OK:
            break
        if got.value > cap:
            cap = int(got.value)
            continue
        raise IOError(lib.acoss_last_error().decode(errors="replace"))
    members = buf[:got.value]
    out = [dict() for _ in range(n)]
    arrays = []
    for m in members:
        shape = tuple(int(m.shape[d]) for d in range(m.ndim))
        a = np.empty(shape, dtype=np.dtype(m.descr.decode()), order="F" if m.fortran else "C")
        arrays.append(a)
        out[m.file][m.name.decode()] = a
    if members:
        dst = (_vp * len(members))(*[a.ctypes.data for a in arrays])
        rc = lib.acoss_npz_read(cpaths, buf, len(members), dst, int(n_threads))
        if rc != ACOSS_OK:
            raise IOError(lib.acoss_last_error().decode(errors="replace"))
    return out


def neg_exp(x):
    """exp(-x) elementwise in the canonical float32 exp (acoss_neg_exp; the early matrix of
    EarlyFusion, earlyfusion_traile.py:182)."""
    torch = _torch()
    lib = load_library()
    X = _dev(x, torch.float32)
    out = torch.empty(X.shape, dtype=torch.float32, device="cuda")
    rc = lib.acoss_neg_exp(_ptr(X), int(X.numel()), _ptr(out), _stream())
    _check(rc, "acoss_neg_exp")
    return out


def snf_step(mats, skip, J, V, reg_diag, out=None, validated=False):
    """One doSimilarityFusionWs cross-diffusion step for matrix `skip`
    (similarity_fusion.py:163-174): S . mean_{m != skip}(mats[m]) . S^T + reg_diag * I.
    mats: list of (n, n) float64 device tensors; J (n, K) column indices, V (n, K) float64
    row-normalised kNN weights of S. Returns a new (n, n) float64 device tensor (or `out`).
    validated=True: J (a device int32 tensor) was checked by `check_knn` already (the fusion loop
    checks each S once, not once per step), so neither the host nor the library checks it again."""
    torch = _torch()
    lib = load_library()
    n = int(mats[0].shape[0])
    for m in mats:
        if m.dtype != torch.float64 or not m.is_cuda or tuple(m.shape) != (n, n) or not m.is_contiguous():
            raise ValueError("snf_step: every matrix must be a contiguous (n, n) float64 device tensor")
    if len(mats) < 2:
        raise ValueError("snf_step: needs at least two matrices (the step averages the others)")
    Jd = _dev(J, torch.int32).contiguous()
    Vd = _dev(V, torch.float64).contiguous()
    if Jd.shape != Vd.shape or Jd.dim() != 2 or Jd.shape[0] != n:
        raise ValueError("snf_step: J and V must both be (n, K)")
    if not validated:
        _check_knn(Jd, n)
    if out is None:
        out = torch.empty((n, n), dtype=torch.float64, device=mats[0].device)
    ptrs = (ctypes.c_void_p * len(mats))(*[m.data_ptr() for m in mats])
    rc = lib.acoss_snf_step(ptrs, len(mats), int(skip), n, _ptr(Jd), _ptr(Vd), int(Jd.shape[1]), float(reg_diag),
                            _ptr(out), 0 if validated else 1, _stream())
    _check(rc, "acoss_snf_step")
    return out


def _knn_dev(J, V, n, validated, what):
    torch = _torch()
    Jd = _dev(J, torch.int32).contiguous()
    Vd = _dev(V, torch.float64).contiguous()
    if Jd.shape != Vd.shape or Jd.dim() != 2 or Jd.shape[0] != n:
        raise ValueError("%s: J and V must both be (n, K)" % what)
    if not validated:
        _check_knn(Jd, n)
    return Jd, Vd


def snf_diffuse_rows(stripes, skip, n, J, V, out=None, validated=False):
    """First half of a row-sharded snf_step (acoss_snf_diffuse_rows): the rows of B = A . S^T
    that belong to this rank's stripe, from the (rows, n) stripes of every matrix. The caller
    all-gathers B's stripes and finishes with snf_left_rows."""
    torch = _torch()
    lib = load_library()
    rows = int(stripes[0].shape[0]) if stripes else 0
    for m in stripes:
        if m.dtype != torch.float64 or not m.is_cuda or tuple(m.shape) != (rows, n) or not m.is_contiguous():
            raise ValueError("snf_diffuse_rows: every stripe must be a contiguous (rows, n) float64 device tensor")
    if len(stripes) < 2:
        raise ValueError("snf_diffuse_rows: needs at least two matrices (the step averages the others)")
    Jd, Vd = _knn_dev(J, V, n, validated, "snf_diffuse_rows")
    if out is None:
        out = torch.empty((rows, n), dtype=torch.float64, device=stripes[0].device)
    ptrs = (ctypes.c_void_p * len(stripes))(*[m.data_ptr() for m in stripes])
    rc = lib.acoss_snf_diffuse_rows(ptrs, len(stripes), int(skip), int(n), rows, _ptr(Jd), _ptr(Vd), int(Jd.shape[1]),
                                    _ptr(out), 0 if validated else 1, _stream())
    _check(rc, "acoss_snf_diffuse_rows")
    return out


def snf_left_rows(B, row0, rows, J, V, reg_diag, out=None, validated=False):
    """Second half of a row-sharded snf_step (acoss_snf_left_rows): rows [row0, row0 + rows) of
    S . B + reg_diag * I from the whole (n, n) B."""
    torch = _torch()
    lib = load_library()
    n = int(B.shape[0])
    if B.dtype != torch.float64 or not B.is_cuda or tuple(B.shape) != (n, n) or not B.is_contiguous():
        raise ValueError("snf_left_rows: B must be a contiguous (n, n) float64 device tensor")
    Jd, Vd = _knn_dev(J, V, n, validated, "snf_left_rows")
    if out is None:
        out = torch.empty((rows, n), dtype=torch.float64, device=B.device)
    rc = lib.acoss_snf_left_rows(_ptr(B), n, int(row0), int(rows), _ptr(Jd), _ptr(Vd), int(Jd.shape[1]),
                                 float(reg_diag), _ptr(out), 0 if validated else 1, _stream())
    _check(rc, "acoss_snf_left_rows")
    return out


def simple_mp_packed(flat, track_off, track_len, pairs, sslen=10, apply_oti=True):
    """SiMPle over packed (12 x n_t) float64 blocks: flat device buffer, element offsets,
    lengths (columns). Returns (score f64 (P,), oti i32 (P,)) device tensors."""
    torch = _torch()
    lib = load_library()
    lens = np.asarray(track_len.cpu() if isinstance(track_len, torch.Tensor) else track_len, np.int64)
    pairs, _ = _pairs_dev(pairs, len(lens))
    P = pairs.shape[0]
    score = torch.empty(P, dtype=torch.float64, device="cuda")
    oti = torch.empty(P, dtype=torch.int32, device="cuda")
    # keep every device buffer referenced until the launch is queued: a temporary passed as
    # _ptr(_dev(...)) returns to torch's caching allocator at once and can be reused
    flat_d = _dev(flat, torch.float64)
    off_d = _dev(track_off, torch.int64)
    len_d = _dev(lens.astype(np.int32), torch.int32)
    rc = lib.acoss_simple_mp(_ptr(flat_d), _ptr(off_d), _ptr(len_d), len(lens), int(lens.max(initial=0)),
                             _ptr(pairs), int(P), int(sslen), int(bool(apply_oti)), _ptr(score), _ptr(oti), _stream())
    _check(rc, "acoss_simple_mp")
    return score, oti


def simple_mp(feats, pairs, sslen=10, apply_oti=True):
    """SiMPle median matrix-profile distance (simple_silva.py:45-118) of ordered pairs.
    feats: list of (12, n) float64 arrays; pairs (P, 2) (query, reference).
    Returns (score f64 (P,), oti i32 (P,)) device tensors; the reference stores -score."""
    torch = _torch()
    mats = [np.asarray(f) if not isinstance(f, torch.Tensor) else f for f in feats]
    for f in mats:
        if f.shape[0] != 12:
            raise ValueError("SiMPle features are (12, n) blocks")
    flat, off, _, cols, _, _ = _pack_mats(mats, torch.float64)
    return simple_mp_packed(flat, off, cols, pairs, sslen, apply_oti)


def median_downsample(feats, track_off, track_len, factor=40):
    """librosa.util.sync(chroma.T, arange(0, n, factor), aggregate=np.median).T per track
    (rqa_serra09.py:44-53). Returns (out (sum ceil(n/f), 12) f32 device, out_off i64, out_len i32)."""
    torch = _torch()
    lib = load_library()
    lens = np.asarray(track_len.cpu() if isinstance(track_len, torch.Tensor) else track_len, np.int64)
    out_len = (lens + factor - 1) // factor
    out_off = np.zeros(len(lens), np.int64)
    if len(lens) > 1:
        out_off[1:] = np.cumsum(out_len[:-1])
    out = torch.empty((max(1, int(out_len.sum())), 12), dtype=torch.float32, device="cuda")
    f = _dev(feats, torch.float32)
    o = _dev(track_off, torch.int64)
    ln = _dev(lens.astype(np.int32), torch.int32)
    oo = _dev(out_off, torch.int64)
    rc = lib.acoss_median_downsample(_ptr(f), _ptr(o), _ptr(ln), len(lens), int(lens.max(initial=0)), int(factor),
                                     _ptr(out), _ptr(oo), _stream())
    _check(rc, "acoss_median_downsample")
    return out[: int(out_len.sum())], out_off, out_len.astype(np.int32)


def hann_smoothing(win_len_smooth=4):
    """Simple.smooth's window: scipy/librosa get_window('hann', L + 2, fftbins=False), sum 1."""
    from scipy import signal
    w = signal.get_window("hann", win_len_smooth + 2, fftbins=False)
    return np.ascontiguousarray(w / np.sum(w), np.float64)


def simple_features(feats, track_off, track_len, win=200, skip=100, win_len_smooth=4):
    """Simple.load_features for every track (simple_silva.py:34-43,56-66).
    Returns (out flat f64 device, out_off i64 (element offsets), T i32 (columns per track));
    track t is out[out_off[t]: out_off[t] + 12*T[t]].view(12, T[t])."""
    torch = _torch()
    lib = load_library()
    lens = np.asarray(track_len.cpu() if isinstance(track_len, torch.Tensor) else track_len, np.int64)
    T = lens // skip
    out_off = np.zeros(len(lens), np.int64)
    if len(lens) > 1:
        out_off[1:] = np.cumsum(12 * T[:-1])
    total = int(12 * T.sum())
    out = torch.empty(max(1, total), dtype=torch.float64, device="cuda")
    w = hann_smoothing(win_len_smooth)
    f = _dev(feats, torch.float32)
    o = _dev(track_off, torch.int64)
    ln = _dev(lens.astype(np.int32), torch.int32)
    oo = _dev(out_off, torch.int64)
    rc = lib.acoss_simple_features(_ptr(f), _ptr(o), _ptr(ln), len(lens), int(win), int(skip),
                                   w.ctypes.data_as(ctypes.c_void_p), len(w), _ptr(out), _ptr(oo), total, _stream())
    _check(rc, "acoss_simple_features")
    return out[:total], out_off, T.astype(np.int32)


def ef_neighbour_error(nb_query, nb_ref, kappa, K):
    """The ValueError the reference raises for a pair of block counts, or None (host-only, no GPU).
    csm_to_binary takes argpartition(D, nn, 1) with nn = round(kappa * ncols) (kappa < 1) or kappa,
    which raises unless nn < ncols (cross_recurrence.py:150-156); getWCSM takes np.partition(CSM, K)
    along the columns and the rows, which raises unless K < ncols and K < nrows
    (similarity_fusion.py:47-50). nb_query / nb_ref: block counts (arrays) of each pair's songs."""
    nq = np.asarray(nb_query, np.int64)
    nr = np.asarray(nb_ref, np.int64)
    if kappa != 0:
        nn = np.round(kappa * nr).astype(np.int64) if kappa < 1 else np.full(nr.shape, int(kappa), np.int64)
        bad = np.flatnonzero(nn >= nr)
        if len(bad):
            b = bad[0]
            return ValueError("kth(=%d) out of bounds (%d)" % (nn[b], nr[b]))
    bad = np.flatnonzero((K >= nr) | (K >= nq))
    if len(bad):
        b = bad[0]
        return ValueError("kth(=%d) out of bounds (%d)" % (K, min(nr[b], nq[b])))
    return None


def _check_ef_neighbours(bank, pairs, kappa, K):
    """Reject pairs whose block counts the reference's argpartition / partition would refuse (see
    ef_neighbour_error) before the kernels run. The smallest counts decide: both conditions are
    monotone in the block count (n - round(kappa n) never decreases with n for kappa < 1)."""
    if isinstance(pairs, np.ndarray):  # host pairs and the bank's host block counts: no sync
        nbp = np.asarray(bank["nb_host"])[pairs]
    else:
        nbp = bank["nb"].long()[pairs.long()]
    lo_q, lo_r = int(nbp[:, 0].min()), int(nbp[:, 1].min())
    err = ef_neighbour_error([lo_q], [lo_r], kappa, K)
    if err is not None:
        raise err


def earlyfusion(bank, pairs, kappa=0.1, K=10, mu=0.5):
    """Batched EarlyFusion scores (earlyfusion_traile.py:157-198). bank: dict of device tensors
    'mfccs', 'ssms', 'chromas' (sum nb x d, float32), 'chroma_med' (T x 12), 'off' (T,) int64,
    'nb' (T,) int32 and host 'max_blocks'. Returns (P, 4) float64 device tensor with columns
    mfccs, ssms, chromas, early."""
    torch = _torch()
    lib = load_library()
    pairs, host = _pairs_dev(pairs, int(bank["nb"].shape[0]))
    P = pairs.shape[0]
    out = torch.empty((P, 4), dtype=torch.float64, device="cuda")
    if P == 0:
        return out
    _check_ef_neighbours(bank, pairs if host is None or "nb_host" not in bank else host, kappa, K)
    T = int(bank["nb"].shape[0])
    order = None
    if P > 4096:
        # pairs in (reference band, query) order: a band of 16 reference tracks' block rows stays
        # cache-resident while every query track's rows stream past it once per band (an i-major
        # pair list streams every reference track's rows once per query). Scores go back to the
        # caller's order. Da-TACOS shape, 15,000 songs: 3.29M -> 4.07M pairs/s (bands of 16..128
        # alike; profiles/r05/ef_short/efband15k_*.log). The runs holding the whole band come
        # first, so they start at multiples of 16 and the CSM kernel's groups of 64 pairs hold
        # four queries with the same 16 references (k_ef_csm_pack packs their rows and columns;
        # profiles/r06/ef_pack/README.txt). No host synchronisation: run lengths by scatter_add.
        band = 16
        key = (pairs[:, 1].to(torch.int64) // band) * T + pairs[:, 0].to(torch.int64)
        order = torch.argsort(key, stable=True)
        ks = key[order]
        start = torch.ones(P, dtype=torch.bool, device=ks.device)
        start[1:] = ks[1:] != ks[:-1]
        rid = torch.cumsum(start, 0) - 1
        runlen = torch.zeros(P, dtype=torch.int64, device=ks.device).scatter_add_(0, rid, torch.ones_like(rid))[rid]
        order = order[torch.argsort((runlen < band).to(torch.int8), stable=True)]
        pairs = pairs[order].contiguous()
    dst = out if order is None else torch.empty_like(out)
    rc = lib.acoss_earlyfusion(_ptr(bank["mfccs"]), _ptr(bank["ssms"]), _ptr(bank["chromas"]), _ptr(bank["chroma_med"]),
                               _ptr(bank["off"]), _ptr(bank["nb"]), T, int(bank["max_blocks"]),
                               int(bank["mfccs"].shape[1]), int(bank["ssms"].shape[1]), int(bank["chromas"].shape[1]),
                               _ptr(pairs), int(P), float(kappa), int(K), float(mu), _ptr(dst), _stream())
    _check(rc, "acoss_earlyfusion")
    if order is not None:
        out[order] = dst
    return out


def ef_block_features(chromas, mfccs, onsets, blocksize=20, mfccs_per_block=50, chromas_per_block=40):
    """EarlyFusion block features of a batch of tracks on the device (acoss_ef_block_features).
    chromas: list of (n_t, 12); mfccs: list of (m_t, d) frame-major (mfcc_htk.T; m_t may differ from
    n_t: the extractor's MFCC frames are longer, features.py:884); onsets: list of frame-index arrays.
    Block b spans mfcc[o[b]:o[b+blocksize-1]] and chroma[o[b]:o[b+blocksize]], each clamped to its
    own length as the reference's slicing (resize_block, earlyfusion_traile.py:240); an empty span
    raises ValueError, as the reference's resize does. NaN MFCCs become 0 (:98). Returns a dict of
    device tensors 'mfccs' (B, R*d), 'ssms' (B, R(R-1)/2), 'chromas' (B, Rc*12), 'chroma_med'
    (T, 12) and host 'block_off' (T,) int64 / 'n_blocks' (T,) int32 (blocks of track t: rows
    block_off[t] .. + n_blocks[t])."""
    torch = _torch()
    lib = load_library()
    T = len(chromas)
    if not (len(mfccs) == len(onsets) == T):
        raise ValueError("one chroma, mfcc and onset array per track")
    n = np.array([len(c) for c in chromas], np.int64)
    nm = np.array([len(m) for m in mfccs], np.int64)
    d = int(np.asarray(mfccs[0]).shape[1]) if T else 20
    nb = np.zeros(T, np.int64)
    for t in range(T):
        o = np.asarray(onsets[t], np.int64)
        if np.asarray(mfccs[t]).ndim != 2 or np.asarray(mfccs[t]).shape[1] != d:
            raise ValueError("track %d: mfcc must be (n_frames, %d) like the first track's" % (t, d))
        if len(o) < blocksize:  # the reference's np.zeros((n_beats - blocksize, ...)) raises here (:106)
            raise ValueError("track %d: %d beats, fewer than blocksize=%d (negative dimensions are not allowed)"
                             % (t, len(o), blocksize))
        nb[t] = len(o) - blocksize
        if nb[t]:
            if o.min() < 0:
                raise ValueError("track %d: negative onset frame" % t)
            b = np.arange(nb[t])
            # the clamped spans of every block (Python slicing); the reference's resize raises on
            # an empty one (skimage.transform.resize of a (0, d) block)
            m1, m2 = np.minimum(o[b], nm[t]), np.minimum(o[b + blocksize - 1], nm[t])
            c1, c2 = np.minimum(o[b], n[t]), np.minimum(o[b + blocksize], n[t])
            if np.any(m2 <= m1) or np.any(c2 <= c1):
                bad = int(np.flatnonzero((m2 <= m1) | (c2 <= c1))[0])
                raise ValueError("track %d: beat block %d spans no frames (onsets %d..%d, %d chroma / %d mfcc "
                                 "frames)" % (t, bad, o[bad], o[bad + blocksize], n[t], nm[t]))
    foff = np.zeros(T, np.int64)
    foff[1:] = np.cumsum(n[:-1])
    moff = np.zeros(T, np.int64)
    moff[1:] = np.cumsum(nm[:-1])
    ooff = np.zeros(T, np.int64)
    ooff[1:] = np.cumsum([len(o) for o in onsets][:-1])
    boff = np.zeros(T, np.int64)
    boff[1:] = np.cumsum(nb[:-1])
    B = int(nb.sum())
    mf = np.concatenate([np.asarray(m, np.float32) for m in mfccs]) if T else np.zeros((0, d), np.float32)
    mf = np.where(np.isnan(mf), np.float32(0), mf)
    ch = np.concatenate([np.asarray(c, np.float32) for c in chromas]) if T else np.zeros((0, 12), np.float32)
    on = np.concatenate([np.asarray(o, np.int64) for o in onsets]) if T else np.zeros(0, np.int64)
    d_mf, d_ch = _dev(mf, torch.float32), _dev(ch, torch.float32)
    d_foff, d_n = _dev(foff, torch.int64), _dev(n.astype(np.int32), torch.int32)
    d_moff, d_nm = _dev(moff, torch.int64), _dev(nm.astype(np.int32), torch.int32)
    d_on, d_ooff, d_boff = _dev(on, torch.int64), _dev(ooff, torch.int64), _dev(boff, torch.int64)
    R, Rc = int(mfccs_per_block), int(chromas_per_block)
    out = {"mfccs": torch.empty((B, R * d), dtype=torch.float32, device="cuda"),
           "ssms": torch.empty((B, R * (R - 1) // 2), dtype=torch.float32, device="cuda"),
           "chromas": torch.empty((B, Rc * 12), dtype=torch.float32, device="cuda"),
           "chroma_med": torch.empty((T, 12), dtype=torch.float32, device="cuda")}
    rc = lib.acoss_ef_block_features(_ptr(d_mf), _ptr(d_ch), _ptr(d_foff), _ptr(d_n), _ptr(d_moff), _ptr(d_nm),
                                     _ptr(d_on), _ptr(d_ooff), _ptr(d_boff), T, B, int(blocksize), R, Rc, d,
                                     _ptr(out["mfccs"]), _ptr(out["ssms"]), _ptr(out["chromas"]),
                                     _ptr(out["chroma_med"]), _stream())
    _check(rc, "acoss_ef_block_features")
    out["block_off"] = boff
    out["n_blocks"] = nb.astype(np.int32)
    return out


FINISH_MODES = {None: 0, "none": 0, "serra09": 1, "chen": 2}


def ds_finish(D, norm=None, symmetric=True, mode=None, out=None):
    """acoss_ds_finish on a (n, n) float32 device matrix: Ds += Ds.T (symmetric) then the
    Serra09 (D / sqrt(n_j)) or Chen (sqrt(n_j) / D) length normalisation with norm[j] =
    sqrt(n_j) in float64. In place unless `out` is given."""
    torch = _torch()
    lib = load_library()
    if D.dtype != torch.float32 or not D.is_cuda or D.dim() != 2 or D.shape[0] != D.shape[1] or D.stride(1) != 1:
        raise ValueError("ds_finish takes a square float32 CUDA matrix with unit column stride")
    m = FINISH_MODES[mode]
    nrm = _dev(norm, torch.float64) if m else None
    if m and nrm.numel() != D.shape[0]:
        raise ValueError("norm must hold one factor per column")
    out = D if out is None else out
    if out.shape != D.shape or out.dtype != D.dtype or out.stride() != D.stride():
        raise ValueError("out must match D")
    rc = lib.acoss_ds_finish(_ptr(D), int(D.shape[0]), int(D.stride(0)), _ptr(nrm), int(bool(symmetric)), m,
                             _ptr(out), _stream())
    _check(rc, "acoss_ds_finish")
    return out


def eval_ranks(D, pos, q_song, m_off, members):
    """acoss_eval_ranks: rank (1-based) of members[m_off[q]:m_off[q+1]] in row q_song[q] of D,
    in np.argsort(-D', 1, kind='stable') order of the clique-permuted matrix (pos = each song's
    position in that order), diagonal -inf. Returns an int32 numpy array."""
    torch = _torch()
    lib = load_library()
    if D.dtype != torch.float32 or not D.is_cuda or D.stride(1) != 1:
        raise ValueError("eval_ranks takes a float32 CUDA matrix with unit column stride")
    n = int(D.shape[0])
    pos = _dev(pos, torch.int32)
    q_song = _dev(q_song, torch.int32)
    m_off = _dev(m_off, torch.int64)
    members = _dev(members, torch.int32)
    for name, t in (("q_song", q_song), ("members", members)):
        if t.numel() and (int(t.min()) < 0 or int(t.max()) >= n):
            raise ValueError("%s must lie in [0, %d)" % (name, n))
    out = torch.empty(members.numel(), dtype=torch.int32, device="cuda")
    rc = lib.acoss_eval_ranks(_ptr(D), n, int(D.stride(0)), _ptr(pos), _ptr(q_song), _ptr(m_off), _ptr(members),
                              int(q_song.numel()), _ptr(out), _stream())
    _check(rc, "acoss_eval_ranks")
    return out.cpu().numpy()


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
