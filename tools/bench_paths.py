"""Throughput of the other scorers on the hot path (SURVEY.md §8a rows beside the headline
metric), each with a CPU baseline timed on the same host in the same run. Informational:
bench.py's JSON line is the metric; this writes one JSON object per path.

    python tools/bench_paths.py [--out profiles/r01/paths.json] [--quick]

Paths:
  serra09_500 / serra09_50: CRP+Qmax at realistic (~500) and short (50) frames per track,
      covers80-shaped corpus; CPU = oracle/crp_oracle.cpp (16 threads) on a sample.
  chen_2000: CRP + Qmax + dmax (ChenFusion) at 2000 frames; CPU = the oracle with dmax.
  simple_200 / simple_2000: SiMPle (OTI + matrix profile + median) on (12 x n) float64
      features, ordered pairs; CPU = oracle.simple_sim (1 thread, direct sums).
  earlyfusion: EarlyFusion.similarity on beat-synchronous block features of 20000-frame
      tracks (~445 blocks; CSMs of 1000/1225/480-d blocks, 4 SW alignments, 3 WCSMs);
      CPU = numpy restatement (oracle/np_oracle.py) + the C SW oracle on a sample.
All inputs synthetic (seeded); GPU timings exclude feature preparation and host transfers.
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

import oracle  # noqa: E402
from oracle import np_oracle as npo  # noqa: E402
from acoss import _lib, synthetic  # noqa: E402
from acoss.engine import ChromaBank  # noqa: E402


def _sync():
    torch.cuda.synchronize()


def crp_path(frames, dmax, reps, cpu_pairs):
    from bench import corpus_tracks
    tracks, _ = corpus_tracks(1, frames, 20250101)
    T = len(tracks)
    pairs = np.array([(i, j) for i in range(T) for j in range(i + 1, T)], np.int32)
    bank = ChromaBank(tracks)
    pt = torch.as_tensor(pairs).cuda()
    bank.crp_align(pt, qmax=True, dmax=dmax)
    _sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = bank.crp_align(pt, qmax=True, dmax=dmax)
    _sync()
    gpu = len(pairs) * reps / (time.perf_counter() - t0)
    feats, off, lens = synthetic.pack(tracks)
    rng = np.random.default_rng(5)
    sp = pairs[rng.choice(len(pairs), size=min(cpu_pairs, len(pairs)), replace=False)]
    nth = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    q, d, _ = oracle.crp_batch(feats, off, lens, sp, dmax=dmax, nthreads=nth)
    cpu = len(sp) / (time.perf_counter() - t0)
    idx = {tuple(p): k for k, p in enumerate(pairs.tolist())}
    sel = [idx[tuple(p)] for p in sp.tolist()]
    ok = bool(np.array_equal(out["qmax"].cpu().numpy()[sel], q))
    if dmax:
        ok = ok and bool(np.array_equal(out["dmax"].cpu().numpy()[sel], d))
    return {"gpu_pairs_per_s": round(gpu, 1), "cpu_pairs_per_s": round(cpu, 2), "cpu_threads": nth,
            "pairs": len(pairs), "frames": frames, "bitexact_vs_oracle": ok, "cpu_sample": len(sp)}


def simple_path(n, n_tracks, reps, cpu_pairs):
    rng = np.random.default_rng(7)
    feats = []
    for _ in range(n_tracks):
        F = np.abs(rng.standard_normal((12, n)))
        feats.append(F / np.linalg.norm(F, axis=0, keepdims=True))
    pairs = np.array([(i, j) for i in range(n_tracks) for j in range(n_tracks) if i != j], np.int32)
    torch_feats = [torch.as_tensor(f).cuda() for f in feats]
    from acoss.synthetic import pack  # noqa: F401
    flat = torch.cat([f.reshape(-1) for f in torch_feats])
    off = np.arange(n_tracks, dtype=np.int64) * 12 * n
    lens = np.full(n_tracks, n, np.int32)
    pt = torch.as_tensor(pairs).cuda()
    _lib.simple_mp_packed(flat, off, lens, pt)
    _sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        score, oti = _lib.simple_mp_packed(flat, off, lens, pt)
    _sync()
    gpu = len(pairs) * reps / (time.perf_counter() - t0)
    sp = pairs[:cpu_pairs]
    t0 = time.perf_counter()
    ref = []
    for i, j in sp:
        k = oracle.simple_oti(feats[i], feats[j])
        ref.append(oracle.simple_sim(feats[i], feats[j], k=k))
    cpu = len(sp) / (time.perf_counter() - t0)
    ok = bool(np.array_equal(score.cpu().numpy()[:len(sp)], np.array(ref)))
    return {"gpu_pairs_per_s": round(gpu, 1), "cpu_pairs_per_s": round(cpu, 2), "cpu_threads": 1,
            "pairs": len(pairs), "frames_per_track": n, "bitexact_vs_oracle": ok, "cpu_sample": len(sp)}


def earlyfusion_path(n_tracks, frames, cpu_pairs, tmp):
    from acoss.algorithms.earlyfusion_traile import EarlyFusion
    tracks, labels = synthetic.make_corpus("covers80", frames=frames, seed=3, stretch=False)
    tracks, labels = tracks[:n_tracks], labels[:n_tracks]
    csv, fdir = synthetic.write_feature_dataset(tmp, tracks, labels, with_mfcc=True)
    ef = EarlyFusion(csv, fdir, shortname="bench", cachedir=os.path.join(tmp, "cache"))
    ef.prepare()
    pairs = np.array([(i, j) for i in range(ef.N) for j in range(i + 1, ef.N)], np.int32)
    for i in range(ef.N):
        ef._device(i)
    ef.similarity(pairs[:8])
    _sync()
    t0 = time.perf_counter()
    ef.similarity(pairs)
    _sync()
    gpu = len(pairs) / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    for i, j in pairs[:cpu_pairs]:
        f1, f2 = ef.load_features(int(i)), ef.load_features(int(j))
        C = [npo.get_csm(f1["mfccs"], f2["mfccs"]), npo.get_csm(f1["ssms"], f2["ssms"]),
             npo.get_csm_blocked_oti(f1["chromas"], f2["chromas"], f1["chroma_med"], f2["chroma_med"],
                                     npo.get_csm_cosine)]
        W = sum(npo.getWCSM(c, ef.K, ef.K) for c in C)
        for B in [npo.csm_to_binary(c, ef.kappa) for c in C] + [npo.csm_to_binary(np.exp(-W), ef.kappa)]:
            oracle.sw_constrained(B)
    cpu = cpu_pairs / (time.perf_counter() - t0)
    nb = ef.load_features(0)["mfccs"].shape[0]
    return {"gpu_pairs_per_s": round(gpu, 2), "cpu_pairs_per_s": round(cpu, 3), "cpu_threads": 1,
            "pairs": len(pairs), "blocks_per_track": int(nb), "cpu_sample": cpu_pairs}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r01", "paths.json"))
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    import tempfile
    q = a.quick
    res = {}
    res["serra09_500"] = crp_path(500, False, 2 if q else 5, 512)
    print(json.dumps({"serra09_500": res["serra09_500"]}), flush=True)
    res["serra09_50"] = crp_path(50, False, 2 if q else 10, 4096)
    print(json.dumps({"serra09_50": res["serra09_50"]}), flush=True)
    res["chen_2000"] = crp_path(2000, True, 2, 96)
    print(json.dumps({"chen_2000": res["chen_2000"]}), flush=True)
    res["simple_200"] = simple_path(200, 64, 2 if q else 5, 64)
    print(json.dumps({"simple_200": res["simple_200"]}), flush=True)
    res["simple_2000"] = simple_path(2000, 64, 1 if q else 2, 4)
    print(json.dumps({"simple_2000": res["simple_2000"]}), flush=True)
    with tempfile.TemporaryDirectory() as tmp:
        res["earlyfusion"] = earlyfusion_path(8 if q else 80, 20000, 4 if q else 8, tmp)
    print(json.dumps({"earlyfusion": res["earlyfusion"]}), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
