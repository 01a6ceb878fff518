"""TEST INFRASTRUCTURE — the EarlyFusion CPU baseline of bench.py. NOT part of the product.

One EarlyFusion.similarity pair (earlyfusion_traile.py:157-198) on the CPU: the numpy
restatement of the three CSMs, csm_to_binary and getWCSM (np_oracle, golden-pinned) and the
C Smith-Waterman of the oracle library. Run as a pool of worker PROCESSES, one interpreter per
core with BLAS held to one thread, so the Python parts of the composition are not serialised on
one interpreter's GIL (a thread pool bought only ~1.5x on 16 threads). The block
features reach the workers as .npy files opened with mmap_mode='r' (no pickling of the banks).
"""
import os

import numpy as np

_BANK = {}


def _init(bank_dir, nb):
    # BLAS / OpenMP at one thread per worker process: the pool provides the parallelism
    for v in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS", "BLIS_NUM_THREADS"):
        os.environ[v] = "1"
    for k in ("mfccs", "ssms", "chromas", "chroma_med"):
        _BANK[k] = np.load(os.path.join(bank_dir, k + ".npy"), mmap_mode="r")
    _BANK["nb"] = int(nb)


def pair_scores(pair, kappa=0.1, K=10):
    """The four scores (mfccs, ssms, chromas, early) of one (i, j) pair of equal-length tracks."""
    import oracle
    from oracle import np_oracle as npo
    i, j = int(pair[0]), int(pair[1])
    nb = _BANK["nb"]

    def feats(t):
        return {k: np.asarray(_BANK[k][t * nb:(t + 1) * nb]) for k in ("mfccs", "ssms", "chromas")}
    f1, f2 = feats(i), feats(j)
    C = [npo.get_csm(f1["mfccs"], f2["mfccs"]), npo.get_csm(f1["ssms"], f2["ssms"]),
         npo.get_csm_blocked_oti(f1["chromas"], f2["chromas"], np.asarray(_BANK["chroma_med"][i]),
                                 np.asarray(_BANK["chroma_med"][j]), npo.get_csm_cosine)]
    W = np.zeros_like(C[0])
    for c in C:
        W += npo.getWCSM(c, K, K)
    return [float(oracle.sw_constrained(npo.csm_to_binary(M, kappa))) for M in C + [np.exp(-W)]]


def run_pool(bank, nb, pairs, nproc, workdir):
    """Scores of `pairs` on `nproc` worker processes (spawned: fresh interpreters that never touch
    the GPU). bank: dict of host arrays mfccs / ssms / chromas (T*nb rows) and chroma_med (T, 12).
    Returns ((P, 4) scores, seconds spent in the pool's map)."""
    import time
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    for k in ("mfccs", "ssms", "chromas", "chroma_med"):
        np.save(os.path.join(workdir, k + ".npy"), np.ascontiguousarray(bank[k]))
    ctx = mp.get_context("spawn")
    with ProcessPoolExecutor(max_workers=nproc, mp_context=ctx, initializer=_init, initargs=(workdir, nb)) as ex:
        list(ex.map(_noop, range(nproc)))  # start every interpreter before the clock
        t0 = time.perf_counter()
        out = list(ex.map(pair_scores, [tuple(p) for p in pairs], chunksize=1))
        dt = time.perf_counter() - t0
    return np.asarray(out, np.float64), dt


def _noop(_):
    import oracle  # noqa: F401  (load the C oracle and numpy in every worker before timing)
    from oracle import np_oracle  # noqa: F401
    return 0
