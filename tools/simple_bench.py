"""SiMPle kernel A/B on the GPU box: pairs/s of acoss_simple_mp at 200 and 2000 frames for the
generic one-thread-per-diagonal kernel (ACOSS_SIMPLE_K=1) and the diagonal-group kernel with
K = 2 / 4 diagonals per lane; every variant's scores checked against the oracle on a sample.

    python tools/simple_bench.py [--out gpurun_out/simple_ab.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "acoss-1_amd"))
sys.path.insert(0, ROOT)
from acoss import _lib  # noqa: E402
import oracle  # noqa: E402


VARIANTS = [("5", "0", "0"), ("4", "0", "1")]  # (K, red, sh[, ppb])


def run(n, n_tracks, reps, check):
    rng = np.random.default_rng(7)
    feats = []
    for _ in range(n_tracks):
        F = np.abs(rng.standard_normal((12, n)))
        feats.append(F / np.linalg.norm(F, axis=0, keepdims=True))
    pairs = np.array([(i, j) for i in range(n_tracks) for j in range(n_tracks) if i != j], np.int32)
    flat = torch.cat([torch.as_tensor(f).cuda().reshape(-1) for f in feats])
    off = np.arange(n_tracks, dtype=np.int64) * 12 * n
    lens = np.full(n_tracks, n, np.int32)
    pt = torch.as_tensor(pairs).cuda()
    ref = []
    for i, j in pairs[:check]:
        k = oracle.simple_oti(feats[i], feats[j])
        ref.append(oracle.simple_sim(feats[i], feats[j], k=k))
    out = {}
    for v in VARIANTS:
        kd, red = v[0], v[1]
        os.environ["ACOSS_SIMPLE_RED"] = red
        os.environ["ACOSS_SIMPLE_SH"] = v[2] if len(v) > 2 else "0"
        if len(v) > 3:
            os.environ["ACOSS_SIMPLE_PPB"] = v[3]
        else:
            os.environ.pop("ACOSS_SIMPLE_PPB", None)
        red = red + ("s" + v[2] if len(v) > 2 else "") + ("p" + v[3] if len(v) > 3 else "")
        os.environ["ACOSS_SIMPLE_K"] = kd
        score, _ = _lib.simple_mp_packed(flat, off, lens, pt)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            score, _ = _lib.simple_mp_packed(flat, off, lens, pt)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        got = score.cpu().numpy()[:check]
        ok = bool(np.array_equal(got, np.array(ref)))
        rel = float(np.max(np.abs(got - np.array(ref)) / np.maximum(np.abs(np.array(ref)), 1e-300)))
        out["K" + kd + "r" + red] = {"pairs_per_s": round(len(pairs) * reps / dt, 1), "bitexact": ok,
                                     "max_rel_diff_vs_oracle": rel}
        print(json.dumps({"n": n, "K": kd, "red": red, **out["K" + kd + "r" + red]}), flush=True)
    os.environ.pop("ACOSS_SIMPLE_K")
    return {"frames": n, "pairs": len(pairs), **out}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "simple_ab.json"))
    ap.add_argument("--frames", type=int, nargs="*", default=[200, 2000])
    ap.add_argument("--variant", default=None, help="K,red (one variant only)")
    a = ap.parse_args()
    global VARIANTS
    if a.variant:
        VARIANTS = [tuple(a.variant.split(","))]
    cfg = {200: (64, 5, 16), 2000: (40, 2, 3), 2001: (100, 1, 3)}
    res = {f"simple_{n}": run(min(n, 2000), *cfg.get(n, (40, 2, 3))) for n in a.frames}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
