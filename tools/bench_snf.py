"""SNF cross-diffusion step throughput (f2): acoss_snf_step on n x n float64 matrices.

    python tools/bench_snf.py [--n 15000] [--L 2] [--K 20] [--reps 5] [--worlds 2,4,8]

Da-TACOS-sized by default (n = 15,000 tracks, K = 20 as LateFusionChen.do_late_fusion,
latefusion_chen.py:88). Times the whole step with HIP events on the launch stream
(rocprofv3 gives the per-kernel split) and prints one JSON line with the step time and the
HBM roofline: algorithmic bytes = (L + 4) * 8 * n^2 (the transpose reads L-1 matrices and
writes one; each of the two gathers reads one matrix, once in the ideal, and writes one).

--worlds: the row-sharded step (similarity_fusion._fusion_sharded) as one rank of W sees it:
acoss_snf_diffuse_rows on a ceil(n/W)-row stripe plus acoss_snf_left_rows of that stripe from
the whole B, timed on this GPU. The all-gather of B between them cannot run on a one-GPU box:
the line gives its bytes per rank and two estimates at the 153 GB/s per xGMI link of an
MI355X node (every peer's stripe on its own link at once; or a ring, W-1 stripes in sequence
over one link).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "acoss-1_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from acoss import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=15000)
    ap.add_argument("--L", type=int, default=2)
    ap.add_argument("--K", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--worlds", default="2,4,8")
    a = ap.parse_args()
    n, L, K = a.n, a.L, a.K
    g = torch.Generator(device="cuda").manual_seed(1)
    mats = [torch.rand((n, n), dtype=torch.float64, device="cuda", generator=g) for _ in range(L)]
    W = torch.rand((n, n), dtype=torch.float32, device="cuda", generator=g)
    V, J = torch.topk(W, K, dim=1)
    V = (V / V.sum(1, keepdim=True)).to(torch.float64)
    J = J.to(torch.int32)
    del W
    out = torch.empty((n, n), dtype=torch.float64, device="cuda")
    _lib.snf_step(mats, 0, J, V, 1.0, out=out)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    for r in range(a.reps):
        e0.record(s)
        _lib.snf_step(mats, r % L, J, V, 1.0, out=out)
        e1.record(s)
        e1.synchronize()
        times.append(e0.elapsed_time(e1))
    ms = float(np.median(times))
    sharded = []
    for w in [int(x) for x in a.worlds.split(",") if x]:
        rows = -(-n // w)
        st = [m[:rows] for m in mats]
        Bfull = torch.empty((n, n), dtype=torch.float64, device="cuda")
        ob = torch.empty((rows, n), dtype=torch.float64, device="cuda")
        _lib.snf_diffuse_rows(st, 0, n, J, V, out=Bfull[:rows], validated=True)
        _lib.snf_left_rows(Bfull, 0, rows, J, V, 1.0, out=ob, validated=True)
        torch.cuda.synchronize()
        tw = []
        for r in range(a.reps):
            e0.record(s)
            _lib.snf_diffuse_rows(st, r % L, n, J, V, out=Bfull[:rows], validated=True)
            _lib.snf_left_rows(Bfull, 0, rows, J, V, 1.0, out=ob, validated=True)
            e1.record(s)
            e1.synchronize()
            tw.append(e0.elapsed_time(e1))
        tms = float(np.median(tw))
        gin = (w - 1) * rows * n * 8.0
        link = 153e9
        sharded.append({"world": w, "rows": rows, "ms_compute": round(tms, 4), "gather_bytes_in": gin,
                        "est_gather_ms_direct": round(rows * n * 8.0 / link * 1e3, 3),
                        "est_gather_ms_ring": round(gin / link * 1e3, 3),
                        "est_step_ms": [round(tms + rows * n * 8.0 / link * 1e3, 3), round(tms + gin / link * 1e3, 3)]})
        del Bfull, ob
    algo = (L + 4) * 8.0 * n * n
    gbs = algo / (ms * 1e-3) / 1e9
    print(json.dumps({"what": "acoss_snf_step (one SNF cross-diffusion step)", "n": n, "L": L, "K": K,
                      "ms_per_step": round(ms, 4), "ms_all": [round(t, 4) for t in times],
                      "algorithmic_bytes": algo, "achieved_GBs": round(gbs, 1), "peak_GBs": 8000.0,
                      "frac": round(gbs / 8000.0, 4),
                      "late_fusion_20_iters_s": round(ms * 20 * L / 1e3, 3), "sharded": sharded}))


if __name__ == "__main__":
    main()
