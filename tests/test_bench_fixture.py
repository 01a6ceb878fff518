"""bench.py's whole-step oracle fixture (tests/golden/bench_oracle_qmax.npz, written by
tests/golden/make_bench_oracle.py) is the oracle's output for exactly the bench corpus (CPU)."""
import hashlib
import os

import numpy as np
import pytest

import oracle
from acoss import synthetic
from conftest import ROOT

FIX = os.path.join(ROOT, "tests", "golden", "bench_oracle_qmax.npz")


@pytest.mark.skipif(not os.path.exists(FIX), reason="fixture not generated")
def test_bench_fixture_matches_corpus_and_oracle():
    with np.load(FIX, allow_pickle=False) as z:
        fx = {k: z[k] for k in z.files}
    frames = int(fx["frames"])
    tracks, labels = synthetic.make_hard_corpus("covers80", frames=frames, seed=int(fx["seed"]))
    h = hashlib.sha256()
    for t in tracks:
        h.update(np.ascontiguousarray(t, np.float32).tobytes())
    assert str(fx["corpus_sha256"]) == h.hexdigest()
    np.testing.assert_array_equal(fx["labels"], labels)
    assert len(fx["qmax"]) == len(fx["pairs"]) == 164 * 163 // 2
    feats, off, lens = synthetic.pack(tracks)
    sel = np.random.default_rng(0).choice(len(fx["pairs"]), 12, replace=False)
    q, _, k = oracle.crp_batch(feats, off, lens, fx["pairs"][sel], dmax=False, nthreads=4)
    np.testing.assert_array_equal(q, fx["qmax"][sel])
    np.testing.assert_array_equal(k, fx["oti"][sel])
