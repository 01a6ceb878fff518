"""One GPU's share of the Da-TACOS configurations (BASELINE.json configs[2..4]).

    python tools/bench_datacos.py [--algo serra09|simple|earlyfusion] [--frames 500] [--world 8]
                                  [--rank 0] [--chunk 1048576] [--max-pairs P]

--algo simple: SiMPle on every ORDERED pair of the stripe (unit-column float64 features of
--frames columns); --algo earlyfusion: the batched EarlyFusion scores of the stripe's pairs on
synthetic block features (--frames beat blocks per track, made on the device); --max-pairs
stops after that many pairs of the stripe (the projection uses the measured rate).

Da-TACOS benchmark-shaped corpus (1000 cliques x 13 + 2000 singletons = 15,000 tracks; synthetic
HPCP, --frames per track at the CSM input, ragged by +-10 %), the cost-balanced row stripe that
rank `--rank` of `--world` GPUs scores (acoss.distributed.stripe_bounds, as all_pairwise does),
scored in PAIR_CHUNK-sized acoss_crp_align calls into a device stripe. Prints progress per chunk
and one JSON line: pairs, seconds, pairs/s, the whole job's projected time on `--world` GPUs, and
(--world 1 only) the device finish + evaluation of the assembled 15,000 x 15,000 matrix.
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

from acoss import _lib, distributed, evaluation, synthetic  # noqa: E402
from acoss.engine import ChromaBank  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=500)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--chunk", type=int, default=1 << 20)
ap.add_argument("--tracks", type=int, default=15000)
ap.add_argument("--algo", choices=["serra09", "simple", "earlyfusion"], default="serra09")
ap.add_argument("--max-pairs", type=int, default=0)
ap.add_argument("--blocks-lo", type=int, default=0,
                help="earlyfusion: ragged beat-block counts, uniform in [--blocks-lo, --frames] per track")
a = ap.parse_args()
t0 = time.perf_counter()
rng = np.random.Generator(np.random.PCG64(20250101))
sizes = synthetic.clique_sizes("datacos")
tracks, labels = [], []
for lab, size in enumerate(sizes):
    n0 = int(round(a.frames * rng.uniform(0.9, 1.1)))
    base = synthetic.base_sequence(rng, n0)
    for v in range(size):
        seq = base if v == 0 else synthetic.cover_of(rng, base, int(round(n0 * rng.uniform(0.9, 1.1))))
        tracks.append(synthetic.render(rng, seq))
        labels.append(lab)
    if len(tracks) >= a.tracks:
        break
tracks, labels = tracks[:a.tracks], np.asarray(labels[:a.tracks], np.int32)
T = len(tracks)
lens = np.array([len(t) for t in tracks], np.int32)
print("corpus: %d tracks, frames %d..%d, %.1f s" % (T, lens.min(), lens.max(), time.perf_counter() - t0), flush=True)
symmetric = a.algo != "simple"
bounds = distributed.stripe_bounds(lens, a.world, symmetric=symmetric)
r0, r1 = bounds[a.rank]
pairs = distributed.stripe_pairs(T, r0, r1, symmetric=symmetric)
if a.max_pairs:
    pairs = pairs[:a.max_pairs]
blk = torch.zeros((r1 - r0, T), dtype=torch.float32, device="cuda")
if a.algo == "serra09":
    bank = ChromaBank(tracks)

    def score(ch):
        return bank.crp_align(ch, qmax=True)["qmax"]
elif a.algo == "simple":
    feats = []
    for t in tracks:
        F = np.ascontiguousarray(np.asarray(t, np.float64).T) + 1e-3
        feats.append(F / np.linalg.norm(F, axis=0, keepdims=True))
    flat = torch.as_tensor(np.concatenate([f.ravel() for f in feats])).cuda()
    off = np.concatenate([[0], np.cumsum([12 * f.shape[1] for f in feats])[:-1]]).astype(np.int64)

    def score(ch):
        sc, _ = _lib.simple_mp_packed(flat, off, lens, ch)
        return (-sc).float()
else:
    NB = a.frames
    nbs = np.full(T, NB, np.int32)
    if a.blocks_lo:
        nbs = np.random.Generator(np.random.PCG64(7)).integers(a.blocks_lo, NB + 1, T).astype(np.int32)
    offs = np.concatenate([[0], np.cumsum(nbs[:-1])]).astype(np.int64)
    R = int(nbs.sum())
    g = torch.Generator(device="cuda").manual_seed(1)
    ebank = {"mfccs": torch.randn((R, 1000), device="cuda", generator=g),
             "ssms": torch.rand((R, 1225), device="cuda", generator=g),
             "chromas": torch.rand((R, 480), device="cuda", generator=g),
             "chroma_med": torch.rand((T, 12), device="cuda", generator=g),
             "off": torch.as_tensor(offs).cuda(), "nb": torch.as_tensor(nbs).cuda(), "nb_host": nbs,
             "max_blocks": int(nbs.max())}

    def score(ch):
        return _lib.earlyfusion(ebank, ch, 0.1, 10)[:, 3].float()
score(pairs[:1024])  # warm the workspaces
torch.cuda.synchronize()
t1 = time.perf_counter()
for c0 in range(0, len(pairs), a.chunk):
    ch = pairs[c0:c0 + a.chunk]
    q = score(ch)
    p = torch.as_tensor(ch.astype(np.int64)).cuda()
    blk[p[:, 0] - r0, p[:, 1]] = q
    torch.cuda.synchronize()
    done = c0 + len(ch)
    el = time.perf_counter() - t1
    print("  %d / %d pairs, %.1f s, %.0f pairs/s" % (done, len(pairs), el, done / el), flush=True)
dt = time.perf_counter() - t1
job = T * (T - 1) // (2 if symmetric else 1)
out = {"algo": a.algo, "tracks": T, "frames": a.frames, "world": a.world, "rank": a.rank, "stripe_rows": [r0, r1],
       "pairs": int(len(pairs)), "seconds": round(dt, 2), "pairs_per_s": round(len(pairs) / dt, 1),
       "job_pairs": job, "projected_job_seconds_on_world": round(job / a.world / (len(pairs) / dt), 1),
       "stripe_checksum": float((blk.double() * (torch.arange(blk.numel(), device="cuda", dtype=torch.float64)
                                                 .reshape(blk.shape) % 7919)).sum())}
if a.world == 1 and not a.max_pairs and a.algo == "serra09":
    norm = np.sqrt(lens.astype(np.float64))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _lib.ds_finish(blk, symmetric=True)
    _lib.ds_finish(blk, norm, symmetric=False, mode="serra09")
    e1.record()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    MR, MRR, MDR, MAP, tops = evaluation.eval_statistics_device(blk, labels=labels)
    out.update({"finish_ms": round(e0.elapsed_time(e1), 3), "eval_s": round(time.perf_counter() - t2, 3),
                "MAP": float(MAP), "MR1": float(MR), "top1": int(tops[0])})
print(json.dumps(out))
