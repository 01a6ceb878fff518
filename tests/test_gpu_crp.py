"""GPU parity: Serra09/Chen CRP + Qmax/dmax (HIP, through the C-ABI) vs the CPU oracle.

Bar (BASELINE.json north_star): OTI index and CRP mask bit-exact; Qmax/dmax exact (the DP
values are multiples of 0.5 in f32); thresholds and distances bit-exact (same canonical
rounding sequence, oracle/crp_oracle.cpp header).
"""
import numpy as np
import pytest

import oracle
from acoss import _lib, synthetic

pytestmark = pytest.mark.gpu


def _pair(rng, M, N):
    base = synthetic.base_sequence(rng, max(M, N))
    X = synthetic.render(rng, base[:M])
    Y = synthetic.render(rng, np.roll(synthetic.cover_of(rng, base, N), 0, 1))
    return X, Y


@pytest.mark.parametrize("M,N,m,tau,oti", [(60, 70, 9, 1, True), (300, 257, 9, 1, True), (523, 611, 9, 2, True),
                                            (200, 180, 4, 1, False), (2000, 2000, 9, 1, True)])
def test_crp_pair_intermediates_bitexact(M, N, m, tau, oti):
    rng = np.random.Generator(np.random.PCG64(M * 1000 + N))
    X, Y = _pair(rng, M, N)
    ref = oracle.crp_pair(X, Y, m=m, tau=tau, kappa=0.095, oti=oti)
    got = _lib.crp_pair(X, Y, _lib.crp_params(m=m, tau=tau, kappa=0.095, oti=oti))
    assert int(got["oti"].item()) == ref["oti"]
    Dref = oracle.crp_dist(X, Y, ref["oti"], m, tau)
    np.testing.assert_array_equal(got["dist"].cpu().numpy().view(np.uint32), Dref.view(np.uint32))
    np.testing.assert_array_equal(got["thr_row"].cpu().numpy().view(np.uint32), ref["thr_row"].view(np.uint32))
    np.testing.assert_array_equal(got["thr_col"].cpu().numpy().view(np.uint32), ref["thr_col"].view(np.uint32))
    np.testing.assert_array_equal(got["crp"].cpu().numpy(), ref["crp"])


def test_crp_align_batch_matches_oracle():
    tracks, labels = synthetic.make_corpus("covers80", frames=300, seed=7)
    tracks = tracks[:24]
    feats, off, lens = synthetic.pack(tracks)
    pairs = np.array([(i, j) for i in range(24) for j in range(i + 1, 24)], np.int32)
    q, d, k = oracle.crp_batch(feats, off, lens, pairs)
    got = _lib.crp_align(feats, off, lens, int(lens.max()), pairs, _lib.crp_params(), qmax=True, dmax=True, oti=True)
    np.testing.assert_array_equal(got["oti"].cpu().numpy(), k)
    np.testing.assert_array_equal(got["qmax"].cpu().numpy(), q)
    np.testing.assert_array_equal(got["dmax"].cpu().numpy(), d)


@pytest.mark.parametrize("M,N,go,ge,align", [(5, 5, 0.5, 0.5, 0), (300, 200, 0.5, 0.5, 0), (300, 200, 0.5, 0.5, 1),
                                             (2100, 90, 0.5, 0.5, 0), (2100, 90, 0.5, 0.5, 1),
                                             (4200, 70, 0.7, 0.3, 0), (4200, 70, 0.7, 0.3, 1),
                                             (257, 4100, 1.0, 0.5, 0),
                                             # the serra09 fast DP (gamma_open == gamma_ext = K/2) at each
                                             # rows-per-lane choice (8 / 16 / 32 and two bands) and K = 0, 2, 3
                                             (300, 200, 0.0, 0.0, 0), (700, 650, 0.5, 0.5, 0),
                                             (1000, 1500, 1.0, 1.0, 0), (2100, 2100, 1.5, 1.5, 0)])
def test_align_crp_matches_oracle(M, N, go, ge, align):
    rng = np.random.Generator(np.random.PCG64(M + 7 * N))
    C = (rng.random((M, N)) < 0.15).astype(np.uint8)
    for t in range(min(M, N)):
        C[t, t] = 1
    ref = oracle.align(C, go, ge, align)
    got = float(_lib.align_crp(C, align, go, ge).item())
    assert got == ref


def test_align_crp_rejects_nonbinary():
    C = np.zeros((10, 10), np.uint8)
    C[3, 4] = 2
    with pytest.raises(_lib.AcossHipError):
        _lib.align_crp(C)


@pytest.mark.parametrize("M,N,silence", [(400, 380, (50, 250)), (2300, 2210, None), (2100, 2300, (100, 700))])
def test_crp_pair_degenerate_rows(M, N, silence):
    """Long silences (huge groups of equal / zero keys) and rows longer than 2048 cells
    exercise the slow exact paths of the threshold select."""
    rng = np.random.Generator(np.random.PCG64(M + N))
    X, Y = _pair(rng, M, N)
    if silence:
        a, b = silence
        X[a:b] = 0.0
        Y[a:b] = 0.0
    ref = oracle.crp_pair(X, Y)
    got = _lib.crp_pair(X, Y, _lib.crp_params())
    np.testing.assert_array_equal(got["thr_row"].cpu().numpy().view(np.uint32), ref["thr_row"].view(np.uint32))
    np.testing.assert_array_equal(got["thr_col"].cpu().numpy().view(np.uint32), ref["thr_col"].view(np.uint32))
    np.testing.assert_array_equal(got["crp"].cpu().numpy(), ref["crp"])


@pytest.mark.parametrize("path", [
    "split", "fused",
    # the alternative kernels the runtime switches select (read once per process, hence the
    # subprocess): generic LDS-Gram select and mask on the fused path, the one-pair-per-wave and
    # the general DP, the f32 chen17 DP instead of the packed one, no lane-strided short lines
    "fused:ACOSS_SELECT_GENERIC=1:ACOSS_MASK_GENERIC=1",
    "split:ACOSS_DP_NOGROUP=1", "split:ACOSS_DP_NOFAST=1", "split:ACOSS_DP_F32=1", "split:ACOSS_NO_SHORT=1"])
def test_crp_align_degenerate_batch(path, monkeypatch):
    """Batch path on silences / ragged lengths / long tracks, both CRP implementations and every
    alternative kernel behind a runtime switch: each equal to the oracle."""
    import subprocess
    import sys
    import os
    code = r'''
import sys, numpy as np
sys.path[:0] = [%r, %r]
import oracle
from acoss import _lib, synthetic
rng = np.random.Generator(np.random.PCG64(99))
tracks = []
for n in [120, 400, 2055, 1500, 37, 900]:
    b = synthetic.base_sequence(rng, n)
    x = synthetic.render(rng, b)
    if n >= 400:
        x[50:300] = 0.0
    tracks.append(x)
feats, off, lens = synthetic.pack(tracks)
pairs = np.array([(i, j) for i in range(len(tracks)) for j in range(len(tracks)) if i != j], np.int32)
q, d, k = oracle.crp_batch(feats, off, lens, pairs)
got = _lib.crp_align(feats, off, lens, int(lens.max()), pairs, _lib.crp_params(), qmax=True, dmax=True, oti=True)
assert np.array_equal(got["oti"].cpu().numpy(), k)
assert np.array_equal(got["qmax"].cpu().numpy(), q), (got["qmax"].cpu().numpy(), q)
assert np.array_equal(got["dmax"].cpu().numpy(), d)
print("ok")
''' % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
       os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "acoss-1_amd"))
    parts = path.split(":")
    env = dict(os.environ, ACOSS_CRP_PATH=parts[0])
    env.update(kv.split("=", 1) for kv in parts[1:])
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_crp_align_run_edges():
    """Split path at line lengths on the 32-element run and 256-column panel edges
    (N' = 32, 33, 289, 1280, 1281, 2016, 2017, 2048): the planes' kNone pads past N' replace the
    selects' tail masks, so every partial run must read as "no element"."""
    rng = np.random.Generator(np.random.PCG64(5))
    tracks = []
    for n in [41, 42, 298, 1289, 1290, 2025, 2026, 2057]:
        x = synthetic.render(rng, synthetic.base_sequence(rng, n))
        if n > 1000:
            x[100:160] = 0.0
        tracks.append(x)
    feats, off, lens = synthetic.pack(tracks)
    pairs = np.array([(i, j) for i in range(len(tracks)) for j in range(len(tracks)) if i != j], np.int32)
    q, d, k = oracle.crp_batch(feats, off, lens, pairs)
    got = _lib.crp_align(feats, off, lens, int(lens.max()), pairs, _lib.crp_params(), qmax=True, dmax=True, oti=True)
    np.testing.assert_array_equal(got["oti"].cpu().numpy(), k)
    np.testing.assert_array_equal(got["qmax"].cpu().numpy(), q)
    np.testing.assert_array_equal(got["dmax"].cpu().numpy(), d)


@pytest.mark.parametrize("lengths", [[10, 41, 42, 73, 74, 137, 300, 521],   # lines <= 512: lane-strided selects
                                     [300, 522, 600, 777, 1000, 1033],  # just past 512: the long-line path
                                     [100, 250, 400, 460, 505],  # DP: 4 pairs per wave (k_crp_dp_grp)
                                     [530, 560, 610, 640, 681]])  # DP: 3 pairs per wave, 20 pairs (not a multiple)
def test_crp_align_short_lines(lengths):
    """Lane-strided selects for batches whose lines all fit 512 codes (element l + 64 q on lane
    l): line ends at every 64-element boundary, a full last lane, silences; and the switch back
    to the long-line path one code later. The short batches also run the grouped Qmax DP
    (several pairs per wave, ragged N' inside a wave, a partly filled last wave)."""
    rng = np.random.Generator(np.random.PCG64(sum(lengths)))
    tracks = []
    for n in lengths:
        x = synthetic.render(rng, synthetic.base_sequence(rng, n))
        if n > 200:
            x[40:130] = 0.0
        tracks.append(x)
    feats, off, lens = synthetic.pack(tracks)
    pairs = np.array([(i, j) for i in range(len(tracks)) for j in range(len(tracks)) if i != j], np.int32)
    q, d, k = oracle.crp_batch(feats, off, lens, pairs)
    got = _lib.crp_align(feats, off, lens, int(lens.max()), pairs, _lib.crp_params(), qmax=True, dmax=True, oti=True)
    np.testing.assert_array_equal(got["oti"].cpu().numpy(), k)
    np.testing.assert_array_equal(got["qmax"].cpu().numpy(), q)
    np.testing.assert_array_equal(got["dmax"].cpu().numpy(), d)


def test_crp_align_long_lines():
    """Lines of 2049..4096 codes (tracks of 2058..4105 frames) stay on the split path: one wave
    holds both 2048-code halves of a line (Line2), mixed in one launch with shorter lines."""
    rng = np.random.Generator(np.random.PCG64(11))
    tracks = []
    for n in [300, 2057, 2058, 2600, 4105]:
        x = synthetic.render(rng, synthetic.base_sequence(rng, n))
        if n > 2000:
            x[1900:2300] = 0.0  # a silence across the halves' boundary
        tracks.append(x)
    feats, off, lens = synthetic.pack(tracks)
    pairs = np.array([(i, j) for i in range(len(tracks)) for j in range(len(tracks)) if i != j], np.int32)
    q, d, k = oracle.crp_batch(feats, off, lens, pairs)
    got = _lib.crp_align(feats, off, lens, int(lens.max()), pairs, _lib.crp_params(), qmax=True, dmax=True, oti=True)
    np.testing.assert_array_equal(got["oti"].cpu().numpy(), k)
    np.testing.assert_array_equal(got["qmax"].cpu().numpy(), q)
    np.testing.assert_array_equal(got["dmax"].cpu().numpy(), d)


def test_crp_align_past_split_limit():
    """A launch with a line of 4097 codes (a 4106-frame track) leaves the split path for the
    generic fused kernels; results stay bit-exact."""
    rng = np.random.Generator(np.random.PCG64(13))
    tracks = [synthetic.render(rng, synthetic.base_sequence(rng, n)) for n in (300, 4106)]
    feats, off, lens = synthetic.pack(tracks)
    pairs = np.array([(0, 1), (1, 0)], np.int32)
    q, d, k = oracle.crp_batch(feats, off, lens, pairs)
    got = _lib.crp_align(feats, off, lens, int(lens.max()), pairs, _lib.crp_params(), qmax=True, dmax=True, oti=True)
    np.testing.assert_array_equal(got["oti"].cpu().numpy(), k)
    np.testing.assert_array_equal(got["qmax"].cpu().numpy(), q)
    np.testing.assert_array_equal(got["dmax"].cpu().numpy(), d)
