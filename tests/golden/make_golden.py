"""Generate the golden vectors under tests/golden/ from the reference itself.

TEST INFRASTRUCTURE. Run in the build container only (it reads /root/reference, which
does not exist on the GPU box):

    python tests/golden/make_golden.py

It imports the reference's pure-Python/numba modules *by file path* with these shims
(none of them changes the arithmetic of the functions captured):

* ``numba.jit`` -> identity decorator (numba is not installed);
* a stub ``acoss`` package (``__path__`` only) so ``acoss/__init__.py`` — which pulls in
  essentia/librosa feature extractors — is never executed;
* empty stubs for ``deepdish``, ``progress.bar`` and ``librosa`` (imported at module
  level by ``algorithm_template.py`` / ``simple_silva.py`` but unused by the captured
  functions).

Captured (reference file:line):
  cross_recurrence.get_ssm/get_csm/get_csm_cosine/get_oti/get_csm_blocked_oti/csm_to_binary
      acoss/algorithms/utils/cross_recurrence.py:10-161
  alignment_tools.smith_waterman_constrained   acoss/algorithms/utils/alignment_tools.py:25-46
  similarity_fusion.getWCSM / doSimilarityFusion  acoss/algorithms/utils/similarity_fusion.py:38-54,188-196
  Simple.oti / Simple.simple_sim               acoss/algorithms/simple_silva.py:45-118
  CoverAlgorithm.getEvalStatistics             acoss/algorithms/algorithm_template.py:206-291

essentia's ChromaCrossSimilarity / CoverSongSimilarity (the Serra09/Chen CRP + Qmax/dmax)
are NOT importable anywhere (no essentia): those rows are pinned by hand-derived
known-answer tests (test_kat_* in tests/test_oracle_golden.py) instead ("parity unpinned" vs
essentia).
"""
import importlib.util
import os
import sys
import tempfile
import types
import contextlib
import io

import numpy as np

REF = "/root/reference/acoss"
OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 20250101


def _stub(name, **attrs):
    mod = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(mod, k, v)
    sys.modules[name] = mod
    return mod


def _load(modname, path):
    spec = importlib.util.spec_from_file_location(modname, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    _stub("numba", jit=lambda *a, **k: (lambda f: f))
    _stub("deepdish", io=types.SimpleNamespace(load=None, save=None))
    _stub("progress")
    _stub("progress.bar", Bar=object)
    _stub("librosa", util=types.SimpleNamespace(), filters=types.SimpleNamespace())
    pkg = _stub("acoss")
    pkg.__path__ = [REF]
    _stub("acoss.utils", create_dataset_filepaths=lambda *a, **k: [])
    alg = _stub("acoss.algorithms")
    alg.__path__ = [REF + "/algorithms"]
    ut = _stub("acoss.algorithms.utils")
    ut.__path__ = [REF + "/algorithms/utils"]
    cr = _load("acoss.algorithms.utils.cross_recurrence", REF + "/algorithms/utils/cross_recurrence.py")
    at = _load("acoss.algorithms.utils.alignment_tools", REF + "/algorithms/utils/alignment_tools.py")
    sf = _load("acoss.algorithms.utils.similarity_fusion", REF + "/algorithms/utils/similarity_fusion.py")
    tpl = _load("acoss.algorithms.algorithm_template", REF + "/algorithms/algorithm_template.py")
    sim = _load("acoss.algorithms.simple_silva", REF + "/algorithms/simple_silva.py")
    return cr, at, sf, tpl, sim


def chroma_like(rng, n, d=12):
    """Non-negative, unit-max per frame (HPCP-like), float32."""
    x = rng.random((n, d)).astype(np.float32) ** 3
    x /= np.maximum(x.max(1, keepdims=True), 1e-6)
    return x.astype(np.float32)


def binary_like(rng, M, N, p):
    B = (rng.random((M, N)) < p).astype(np.uint8)
    # add a few diagonal runs so the alignment scores are non-trivial
    for _ in range(max(1, (M * N) // 2000)):
        i0, j0 = rng.integers(0, M), rng.integers(0, N)
        L = int(rng.integers(3, 40))
        for t in range(L):
            if i0 + t < M and j0 + t < N:
                B[i0 + t, j0 + t] = 1
    return B


def main():
    cr, at, sf, tpl, sim = load_reference()
    rng = np.random.Generator(np.random.PCG64(SEED))
    out = {}

    # --- get_csm / get_csm_cosine / get_ssm (cross_recurrence.py:10-73) ---
    for tag, (M, N, d) in {"s": (50, 60, 12), "m": (200, 180, 108)}.items():
        X = rng.standard_normal((M, d)).astype(np.float32)
        Y = rng.standard_normal((N, d)).astype(np.float32)
        Y[3] = 0.0  # zero-norm row exercises the cosine guard (:68-70)
        out[f"csm_{tag}_X"], out[f"csm_{tag}_Y"] = X, Y
        out[f"csm_{tag}_euclid"] = cr.get_csm(X, Y)
        out[f"csm_{tag}_cosine"] = cr.get_csm_cosine(X, Y)
        out[f"ssm_{tag}"] = cr.get_ssm(X)

    # --- get_oti (cross_recurrence.py:75-103), incl. a constructed tie ---
    C1s, C2s, otis = [], [], []
    for t in range(24):
        c1 = rng.random(12).astype(np.float32)
        k = t % 12
        c2 = np.roll(c1, k) + 0.05 * rng.random(12).astype(np.float32)
        C1s.append(c1); C2s.append(c2.astype(np.float32))
    tie = np.array([1, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0], np.float32)  # shifts 0 and 6 tie
    C1s.append(tie); C2s.append(tie.copy())
    for c1, c2 in zip(C1s, C2s):
        otis.append(int(cr.get_oti(c1, c2)))
    out["oti_C1"], out["oti_C2"], out["oti_idx"] = np.stack(C1s), np.stack(C2s), np.array(otis, np.int32)

    # --- get_csm_blocked_oti with cosine (cross_recurrence.py:105-134): 480-d blocks ---
    Xb = rng.random((40, 480)).astype(np.float32)
    Yb = rng.random((50, 480)).astype(np.float32)
    c1 = np.median(Xb.reshape(-1, 12), 0).astype(np.float32)
    c2 = np.median(Yb.reshape(-1, 12), 0).astype(np.float32)
    out["boti_X"], out["boti_Y"], out["boti_C1"], out["boti_C2"] = Xb, Yb, c1, c2
    out["boti_cosine"] = cr.get_csm_blocked_oti(Xb, Yb, c1, c2, cr.get_csm_cosine)
    out["boti_euclid"] = cr.get_csm_blocked_oti(Xb, Yb, c1, c2, cr.get_csm)

    # --- csm_to_binary (cross_recurrence.py:136-161), tie-free inputs ---
    D = rng.permutation(60 * 70).reshape(60, 70).astype(np.float32) / 100.0
    out["bin_D"] = D
    for kap, tag in [(0.0, "k0"), (0.095, "k0095"), (0.1, "k01"), (5, "k5")]:
        out[f"bin_{tag}"] = np.asarray(cr.csm_to_binary(D, kap)).astype(np.uint8)
    # a tie case: all-zero rows against 5 tied zero columns; record the reference's choice
    Dt = np.ones((4, 20), np.float32)
    Dt[:, [2, 5, 7, 11, 13]] = 0.0
    out["bin_tie_D"] = Dt
    out["bin_tie_k3"] = np.asarray(cr.csm_to_binary(Dt, 3)).astype(np.uint8)

    # --- smith_waterman_constrained (alignment_tools.py:25-46) ---
    sw_shapes = [(3, 10), (4, 4), (5, 7), (30, 40), (100, 120), (64, 300), (300, 300)]
    for n, (M, N) in enumerate(sw_shapes):
        p = [0.1, 0.5, 0.2, 0.1, 0.08, 0.12, 0.1][n]
        B = binary_like(rng, M, N, p)
        out[f"sw_{n}_B"] = B
        out[f"sw_{n}_score"] = np.float64(at.smith_waterman_constrained(B))

    # --- getWCSM (similarity_fusion.py:38-54) ---
    CSM = (rng.random((50, 60)) * 2).astype(np.float32)
    out["wcsm_CSM"] = CSM
    out["wcsm_W"] = sf.getWCSM(CSM, 10, 10)

    # --- doSimilarityFusion (similarity_fusion.py:188-196), N=40, 3 matrices ---
    Ds = []
    for _ in range(3):
        A = rng.random((40, 40))
        Ds.append((A + A.T) / 2)
    out["snf_D"] = np.stack(Ds)
    out["snf_fused"] = sf.doSimilarityFusion(Ds, K=5, niters=5, reg_diag=1)[1]

    # --- Simple.oti + simple_sim (simple_silva.py:45-118) ---
    S = sim.Simple.__new__(sim.Simple)
    S.SSLEN = 10
    for tag, (na, nb) in {"a": (20, 20), "b": (200, 180), "c": (2000, 2000)}.items():
        A = rng.random((12, na))
        Bm = rng.random((12, nb))
        A /= np.linalg.norm(A, axis=0, keepdims=True)
        Bm /= np.linalg.norm(Bm, axis=0, keepdims=True)
        Bo, sidx = S.oti(A, Bm)
        out[f"simple_{tag}_A"], out[f"simple_{tag}_B"] = A, Bm
        out[f"simple_{tag}_oti"] = np.int32(sidx[-1])
        out[f"simple_{tag}_Brot"] = Bo
        out[f"simple_{tag}_score"] = np.float64(S.simple_sim(A, Bo))

    # --- getEvalStatistics (algorithm_template.py:206-291) ---
    cov = np.genfromtxt(REF + "/data/covers80_annotations.csv", delimiter=",", dtype=str, skip_header=1)
    labels80 = cov[:, 0]
    _, lab80 = np.unique(labels80, return_inverse=True)
    lab_dt = np.concatenate([np.repeat(np.arange(20), 13), 20 + np.arange(40)])
    for tag, lab in {"c80": lab80, "dt": lab_dt}.items():
        N = len(lab)
        Dm = rng.random((N, N)).astype(np.float32)
        Dm[lab[:, None] == lab[None, :]] += 0.35  # make covers closer, tie-free
        alg = tpl.CoverAlgorithm.__new__(tpl.CoverAlgorithm)
        alg.name, alg.shortname = "Golden", tag
        alg.Ds = {"main": Dm}
        alg.cliques = {}
        for i, l in enumerate(lab):
            alg.cliques.setdefault(str(l), set()).add(i)
        with tempfile.TemporaryDirectory() as td, contextlib.redirect_stdout(io.StringIO()):
            cwd = os.getcwd()
            os.chdir(td)
            try:
                MR, MRR, MDR, MAP, tops = alg.getEvalStatistics("main")
                csv_text = open("results_%s_Golden.csv" % tag).read()
            finally:
                os.chdir(cwd)
        out[f"eval_{tag}_D"], out[f"eval_{tag}_labels"] = Dm, lab.astype(np.int32)
        out[f"eval_{tag}_stats"] = np.array([MR, MRR, MDR, MAP], np.float64)
        out[f"eval_{tag}_tops"] = np.asarray(tops, np.float64)
        out[f"eval_{tag}_csv"] = np.array(csv_text)

    np.savez_compressed(os.path.join(OUT, "reference_golden.npz"), **out)
    print("wrote", os.path.join(OUT, "reference_golden.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
