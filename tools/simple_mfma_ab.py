"""SiMPle A/B on the GPU box: the MFMA kernel (k_simple_mfma, frame dots on v_mfma_f64_16x16x4_f64)
against the VALU diagonal-group kernels (ACOSS_SIMPLE_MFMA=0), same inputs, same process (the
switch is read per call). Scores of both must be identical, and equal to the oracle on a sample.

    python tools/simple_mfma_ab.py [--out gpurun_out/simple_mfma_ab.json]

Cases: every ordered pair of N unit-column tracks of fixed length (200, 500, 2000 frames, the bench
leg's 2000 among them) and of Da-TACOS-like ragged lengths (350..700 frames).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "acoss-1_amd")]
from acoss import _lib  # noqa: E402
import oracle  # noqa: E402


def case(lengths, reps, check, seed=7):
    rng = np.random.default_rng(seed)
    feats = []
    for n in lengths:
        F = np.abs(rng.standard_normal((12, int(n)))) + 1e-3
        feats.append(F / np.linalg.norm(F, axis=0, keepdims=True))
    T = len(feats)
    pairs = np.array([(i, j) for i in range(T) for j in range(T) if i != j], np.int32)
    flat = np.concatenate([f.ravel() for f in feats])
    lens = np.array([f.shape[1] for f in feats], np.int32)
    off = np.concatenate([[0], np.cumsum(12 * lens[:-1].astype(np.int64))]).astype(np.int64)
    fd, pt = torch.as_tensor(flat).cuda(), torch.as_tensor(pairs).cuda()
    out = {"tracks": T, "pairs": int(len(pairs)), "frames": [int(lens.min()), int(lens.max())]}
    scores = {}
    for tag, env in (("mfma", "1"), ("valu", "0")):
        os.environ["ACOSS_SIMPLE_MFMA"] = env
        _lib.simple_mp_packed(fd, off, lens, pt)
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            sc, _ = _lib.simple_mp_packed(fd, off, lens, pt)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = float(np.median(ts))
        scores[tag] = sc.cpu().numpy()
        cells = float(np.sum((lens[pairs[:, 0]] - 9).astype(np.float64) * (lens[pairs[:, 1]] - 9)))
        ops = float(np.sum(24.0 * lens[pairs[:, 0]].astype(np.float64) * lens[pairs[:, 1]])) + 16.0 * cells
        out[tag] = {"ms": round(ms, 3), "pairs_per_s": round(len(pairs) / (ms * 1e-3), 1),
                    "frac_f64": round(ops / (ms * 1e-3) / 1e12 / 78.6, 4)}
    os.environ.pop("ACOSS_SIMPLE_MFMA", None)
    out["identical"] = bool(np.array_equal(scores["mfma"], scores["valu"]))
    idx = np.random.default_rng(seed + 1).choice(len(pairs), min(check, len(pairs)), replace=False)
    cs, _ = oracle.simple_batch(flat, off, lens, pairs[idx], nthreads=16)
    out["oracle_equal"] = "%d of %d" % (int(np.sum(scores["mfma"][idx] == cs)), len(idx))
    out["speedup"] = round(out["valu"]["ms"] / out["mfma"]["ms"], 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = {}
    rng = np.random.default_rng(3)
    for name, lengths, reps, check in (("200", [200] * 120, 3, 300), ("500", [500] * 120, 3, 200),
                                        ("2000", [2000] * 80, 3, 60),
                                        ("350-700", rng.integers(350, 701, size=150), 3, 200)):
        res[name] = case(lengths, reps, check)
        print(name, json.dumps(res[name]), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
