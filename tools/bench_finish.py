"""Time the device finish and evaluation at Da-TACOS shape on one GPU.

    python tools/bench_finish.py [--n 15000] [--host]

A synthetic (n x n) float32 upper-triangle score matrix with the Da-TACOS benchmark clique
structure (1000 cliques of 13 + 2000 singletons at n = 15,000): acoss_ds_finish (Ds += Ds.T, then
Serra09's / sqrt(n_j)) and evaluation.eval_statistics_device (acoss_eval_ranks + the O(N) host
statistics), each timed with HIP events / wall clock; --host also times the reference-order
numpy path (D + D.T, / sqrt, eval_statistics) and checks that the two agree exactly.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "acoss-1_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from acoss import _lib, evaluation, synthetic  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=15000)
ap.add_argument("--host", action="store_true")
a = ap.parse_args()
sizes = synthetic.clique_sizes("datacos")
labels = np.concatenate([np.full(s, c) for c, s in enumerate(sizes)])[: a.n]
n = len(labels)
rng = np.random.default_rng(1)
D = np.triu(rng.random((n, n), dtype=np.float32) * 40, 1)
same = labels[:, None] == labels[None, :]
D[np.triu(same, 1)] += 25.0  # covers score higher, with overlap
norm = np.sqrt(rng.integers(300, 700, size=n).astype(np.float64))
out = {"n": n, "cliques": int(len(np.unique(labels)))}
Dg = torch.as_tensor(D).cuda()
torch.cuda.synchronize()
for rep in range(3):
    X = Dg.clone()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    _lib.ds_finish(X, symmetric=True)
    e1.record()
    _lib.ds_finish(X, norm, symmetric=False, mode="serra09")
    e2.record()
    torch.cuda.synchronize()
    out["ds_finish_sym_ms"] = round(e0.elapsed_time(e1), 3)
    out["ds_finish_norm_ms"] = round(e1.elapsed_time(e2), 3)
    out["ds_finish_GBps"] = round(2 * 2 * 4 * n * n / (e0.elapsed_time(e2) * 1e-3) / 1e9, 1)
    t0 = time.perf_counter()
    stats = evaluation.eval_statistics_device(X, labels=labels)
    torch.cuda.synchronize()
    out["eval_device_s"] = round(time.perf_counter() - t0, 3)
out["MAP"] = float(stats[3])
out["MR1"] = float(stats[0])
if a.host:
    t0 = time.perf_counter()
    H = (D + D.T)
    H = (H / norm[None, :]).astype(np.float32)
    out["host_finish_s"] = round(time.perf_counter() - t0, 3)
    out["finish_bitexact"] = bool(np.array_equal(H, X.cpu().numpy()))
    t0 = time.perf_counter()
    hs = evaluation.eval_statistics(H, labels)
    out["eval_host_s"] = round(time.perf_counter() - t0, 3)
    out["eval_identical"] = bool(all(x == y for x, y in zip(hs[:4], stats[:4])) and np.array_equal(hs[4], stats[4]))
print(json.dumps(out))
