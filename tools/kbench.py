"""Run acoss_crp_align once on the bench corpus (for rocprof / ablation runs).

    python tools/kbench.py [--pairs N] [--frames F] [--reps R]
Prints per-phase HIP-event times (ms per launch).
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "acoss-1_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from acoss import _lib  # noqa: E402
from acoss.engine import ChromaBank  # noqa: E402
from bench import corpus_tracks  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pairs", type=int, default=4000)
ap.add_argument("--frames", type=int, default=2000)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--dmax", action="store_true")
ap.add_argument("--noprof", action="store_true", help="no per-phase events: plain wall time per call")
ap.add_argument("--corpus", choices=["hard", "bench"], default="hard")
ap.add_argument("--mixed", default="", help="LO,HI: each track cut to a length drawn from [LO, HI] (HI <= frames)")
a = ap.parse_args()
tracks, labels = corpus_tracks(1, a.frames, 20250101, a.corpus)
if a.mixed:
    lo, hi = (int(v) for v in a.mixed.split(","))
    rng = np.random.Generator(np.random.PCG64(7))
    tracks = [t[: int(rng.integers(lo, hi + 1))] for t in tracks]
bank = ChromaBank(tracks)
T = len(tracks)
pairs = np.array([(i, j) for i in range(T) for j in range(i + 1, T)], np.int32)[: a.pairs]
pt = torch.as_tensor(pairs).cuda()
for r in range(a.reps):
    _lib.profile_enable(not a.noprof)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = bank.crp_align(pt, qmax=True, dmax=a.dmax)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ph = {} if a.noprof else _lib.profile_read()
    _lib.profile_enable(False)
    print("rep %d: %.1f pairs/s  %s" % (r, len(pairs) / dt, {k: round(v[0] / v[1], 3) for k, v in ph.items()}))
print("qmax checksum", float(out["qmax"].double().sum()))
