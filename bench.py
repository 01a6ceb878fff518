#!/usr/bin/env python
"""bench.py — song-pairs/s of the Serra09 hot path (OTI -> CRP -> Qmax) on MI355X.

Metric (BASELINE.json): "song-pairs/sec (CSM+Qmax) on 12-d HPCP, ~2000 frames/track; MAP parity".
Workload (configs[1]): covers80-shaped corpus (164 tracks: 77x2, 2x3, 1x4 cliques), synthetic
12-d HPCP, every track exactly 2000 frames at the CSM input (M = N = 2000, M' = N' = 1991),
essentia defaults m=9, tau=1, kappa=0.095, OTI on, gamma 0.5/0.5. A step = every unordered
pair (i < j) of the corpus scored once = 13,366 pairs at N=1. Features are resident in HBM
before the timed region. The default corpus is the discriminative one (synthetic.make_hard_corpus:
shared chord phrases, partial re-harmonised covers; MAP about 0.8 at 2000 frames), so the MAP/MR1
comparison against the oracle can fail; --corpus bench is the round-1/2 corpus (MAP 1.0).

Multi-GPU (one process per GPU, torchrun): weak scaling. The corpus grows to
round(164 * sqrt(N)) tracks (the covers80 clique pattern repeated), so each rank scores a
cost-balanced row stripe of ~13.4k pairs; each step ends with ONE all-gather of the stripes
(RCCL over xGMI) that assembles the full N x N score matrix on every rank. value = all
pairs of all ranks / max-over-ranks time.

Also reported: roofline of the path (SURVEY.md §8d ops_pair) with per-kernel HIP-event
times, MAP/MR1 of the assembled matrix (reference normalisation + evaluation), and the CPU
baseline: the oracle (C++ restatement, oracle/) timed on the host cores of this node over a
bounded random sample of the same pairs, whose Qmax values are also checked for equality.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "acoss-1_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

PEAK_F32_TFLOPS = 157.3  # MI355X fp32 (matrix = vector) dense peak, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0


def ops_pair(M, N, m=9, tau=1):
    """2*12*M*N (Gram) + 32*M'*N' (window, norms, sqrt, thresholds, DP)."""
    Mp = max(0, -(-(M - m * tau) // tau))
    Np = max(0, -(-(N - m * tau) // tau))
    return 2.0 * 12 * M * N + 32.0 * Mp * Np


# SURVEY.md §8d's 32 ops per CRP cell split by the kernel that does them: the sweep (Gram 2*12
# per frame pair, 8 window adds, 2 norm terms, 1 sqrt), the two line selects and the mask (2
# compares, 1 AND, 4 select), the DP (14).
def ops_split(M, N, m=9, tau=1):
    Mp = max(0, -(-(M - m * tau) // tau))
    Np = max(0, -(-(N - m * tau) // tau))
    cells = float(Mp * Np)
    return {"sweep": 2.0 * 12 * M * N + 11.0 * cells, "selects": 7.0 * cells, "dp": 14.0 * cells}


# library phase -> its share of ops_split (the fused row select runs inside the sweep kernel, so
# the "sweep" phase carries the sweep's ops and half of the selects' ops; "select_cols" the rest)
PHASE_OPS = {"sweep": lambda s: s["sweep"] + 0.5 * s["selects"], "select_cols": lambda s: 0.5 * s["selects"],
             "dp_qmax": lambda s: s["dp"]}


def build_id():
    """Identity of the HIP build this tree runs: SHA-256 (first 16 hex) of the kernel sources and
    their Makefile (acoss-1_amd/csrc, include/), and of the built library. profiles/profile.sh
    records the same ids next to the counters, so bench.py can refuse PMC figures measured on
    another build."""
    import glob
    import hashlib
    h = hashlib.sha256()
    srcs = sorted(glob.glob(os.path.join(ROOT, "acoss-1_amd", "csrc", "*")) + glob.glob(os.path.join(ROOT, "include", "*.h")))
    for f in srcs:
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    lib = os.path.join(ROOT, "acoss-1_amd", "acoss", "lib", "libacoss_hip.so")
    lh = None
    if os.path.exists(lib):
        with open(lib, "rb") as fh:
            lh = hashlib.sha256(fh.read()).hexdigest()[:16]
    return {"src_sha16": h.hexdigest()[:16], "lib_sha16": lh}


def log(msg):
    """Progress on stderr (the JSON line is the only stdout output)."""
    print("[bench %.1fs] %s" % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


T_START = time.perf_counter()


def cgroup_cpu_quota():
    """CPUs the cgroup's CFS quota grants this process (cgroup v2 cpu.max or v1
    cpu.cfs_quota_us / cpu.cfs_period_us), None when unlimited or unreadable, and the source."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            return (None if q == "max" else float(q) / float(per)), path
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return (None if q <= 0 else q / per), "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"
    except (OSError, ValueError):
        return None, None


def cpu_share():
    """(threads, how they were chosen) for the CPU baselines: every CPU the box grants this
    process. A CFS quota, when there is one, bounds the affinity mask; without one the box's
    per-GPU CPU share is what it exports as OMP_NUM_THREADS (nproc and the affinity mask there
    show the whole machine); else every CPU in the affinity mask."""
    n = len(os.sched_getaffinity(0))
    quota, _ = cgroup_cpu_quota()
    if quota:
        return max(1, min(n, int(math.floor(quota)))), "cgroup CFS quota"
    try:
        omp = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        omp = 0
    if 0 < omp < n:
        return omp, "OMP_NUM_THREADS (the box's per-GPU CPU share; no CFS quota set)"
    return n, "sched_getaffinity"


ORACLE_FIXTURE = os.path.join(ROOT, "tests", "golden", "bench_oracle_qmax.npz")


def oracle_map_parity(tracks, labels, lens, pairs, Dfull, Dsym, frames, gpu_stats):
    """The whole step against the oracle: the oracle's Qmax for every pair of this corpus
    (tests/golden/make_bench_oracle.py; a full oracle step takes ~20 min on the box's 16-thread
    share, so it is precomputed for this exact corpus), compared bit for bit with the GPU's, and
    MR/MRR/MDR/MAP/Top-k of both finished matrices (algorithm_template.py:206-291)."""
    from acoss import evaluation
    if not os.path.exists(ORACLE_FIXTURE):
        return {"error": "no oracle fixture (tests/golden/make_bench_oracle.py)"}
    import hashlib
    with np.load(ORACLE_FIXTURE, allow_pickle=False) as z:
        fx = {k: z[k] for k in z.files}
    h = hashlib.sha256()
    for t in tracks:
        h.update(np.ascontiguousarray(t, np.float32).tobytes())
    if int(fx["frames"]) != frames or str(fx["corpus_sha256"]) != h.hexdigest() or \
            not np.array_equal(fx["pairs"], pairs):
        return {"error": "oracle fixture is for another corpus/length"}
    q = fx["qmax"]
    gq = Dfull[pairs[:, 0], pairs[:, 1]].astype(np.float32)
    Do = np.zeros_like(Dfull)
    Do[pairs[:, 0], pairs[:, 1]] = q
    Dos = (Do + Do.T).astype(np.float32)
    Dos = (Dos / np.sqrt(lens.astype(np.float64))[None, :]).astype(np.float32)
    oMR, oMRR, oMDR, oMAP, otops = evaluation.eval_statistics(Dos, labels)
    MR, MRR, MDR, MAP, tops = gpu_stats
    st = lambda a, b, c, d, e: {"MAP": float(d), "MR1": float(a), "MRR": float(b), "MDR": float(c),  # noqa: E731
                                "top": [int(t) for t in e]}
    same = bool(np.array_equal(Dos, Dsym) and MAP == oMAP and MR == oMR and MRR == oMRR and MDR == oMDR
                and np.array_equal(tops, otops))
    return {"pairs_compared": int(len(q)), "qmax_pairs_differing": int(np.sum(gq != q)),
            "gpu": st(MR, MRR, MDR, MAP, tops), "oracle": st(oMR, oMRR, oMDR, oMAP, otops),
            "ds_bitexact": bool(np.array_equal(Dos, Dsym)), "identical": same,
            "oracle_source": "tests/golden/bench_oracle_qmax.npz (oracle/crp_oracle.cpp, every pair)"}


PEAK_F64_TFLOPS = 78.6  # MI355X fp64 vector dense peak, MI355X_MICROARCH.md


def other_paths(nth, seed):
    """The other scorers on the path on one GPU, each timed with HIP events
    on its launch stream beside a CPU oracle sample of the same inputs:
      simple: SiMPle (Simple.oti + matrix profile + median, simple_silva.py:45-126) on every ORDERED
        pair of 164 tracks x 2000 columns of unit-column float64 features (the covers80-shaped hard
        corpus as SiMPle features); ops/pair = 2*12*na*nb + 16*(na-9)*(nb-9), f64 VALU.
      earlyfusion: EarlyFusion.similarity (earlyfusion_traile.py:157-198) batched over every pair of
        80 tracks x 446 beat blocks (synthetic block features); flops/pair = 2*(1000+1225+480)*M*N
        on the fp32 MFMA CSMs, plus 4 SW and 3 WCSMs.
      snf: one SNF cross-diffusion step at Da-TACOS size (snf_path).
      datacos_stripe: config 3's per-GPU share, Serra09 on rank 0's stripe of the 8-GPU Da-TACOS split
        (datacos_stripe).
    """
    import torch
    import oracle
    from acoss import _lib, synthetic
    res = {}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # ---- SiMPle
    tracks, _ = synthetic.make_hard_corpus("covers80", frames=2000, seed=seed)
    feats = []
    for t in tracks:
        F = np.ascontiguousarray(np.asarray(t, np.float64).T) + 1e-3
        feats.append(F / np.linalg.norm(F, axis=0, keepdims=True))
    T = len(feats)
    n = feats[0].shape[1]
    flat = np.concatenate([f.ravel() for f in feats])
    off = np.arange(T, dtype=np.int64) * 12 * n
    lens = np.full(T, n, np.int32)
    pairs = np.array([(i, j) for i in range(T) for j in range(T) if i != j], np.int32)
    flat_d, pt = torch.as_tensor(flat).cuda(), torch.as_tensor(pairs).cuda()
    _lib.simple_mp_packed(flat_d, off, lens, pt)
    torch.cuda.synchronize()
    ev0.record()
    score, _ = _lib.simple_mp_packed(flat_d, off, lens, pt)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1)
    ops = 2.0 * 12 * n * n + 16.0 * (n - 9) * (n - 9)
    sp = pairs[np.random.Generator(np.random.PCG64(3)).choice(len(pairs), 960, replace=False)]
    t0 = time.perf_counter()
    cs, _ = oracle.simple_batch(flat, off, lens, sp, nthreads=nth)
    cdt = time.perf_counter() - t0
    g = score.cpu().numpy()
    idx = sp[:, 0] * (T - 1) + sp[:, 1] - (sp[:, 1] > sp[:, 0])
    res["simple"] = {"metric": "ordered song-pairs/s (SiMPle matrix profile, 2000 columns)",
                     "value": round(len(pairs) / (ms * 1e-3), 1), "ms": round(ms, 3), "pairs": int(len(pairs)),
                     "dtype": "f64",
                     "roofline": {"bound": "valu", "achieved": round(ops * len(pairs) / (ms * 1e-3) / 1e12, 3),
                                  "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s",
                                  "frac": round(ops * len(pairs) / (ms * 1e-3) / 1e12 / PEAK_F64_TFLOPS, 4),
                                  "ops_per_pair": ops},
                     "cpu_baseline": {"value": round(len(sp) / cdt, 3), "cores": nth, "kind": "port",
                                      "sample": "%d ordered pairs, oracle or_simple_batch, %.1f s" % (len(sp), cdt)},
                     "bitexact_vs_oracle": bool(np.array_equal(g[idx], cs))}
    # ---- EarlyFusion
    rng = np.random.Generator(np.random.PCG64(seed))
    NT, NB = 80, 446
    mf = rng.standard_normal((NT * NB, 1000), dtype=np.float32)
    ss = np.abs(rng.standard_normal((NT * NB, 1225), dtype=np.float32))
    ch = np.abs(rng.standard_normal((NT * NB, 480), dtype=np.float32))
    med = np.abs(rng.standard_normal((NT, 12), dtype=np.float32))
    bank = {"mfccs": torch.as_tensor(mf).cuda(), "ssms": torch.as_tensor(ss).cuda(), "chromas": torch.as_tensor(ch).cuda(),
            "chroma_med": torch.as_tensor(med).cuda(),
            "off": torch.as_tensor(np.arange(NT, dtype=np.int64) * NB).cuda(),
            "nb": torch.as_tensor(np.full(NT, NB, np.int32)).cuda(), "max_blocks": NB}
    epairs = np.array([(i, j) for i in range(NT) for j in range(i + 1, NT)], np.int32)
    _lib.earlyfusion(bank, epairs[:64], 0.1, 10)
    torch.cuda.synchronize()
    ev0.record()
    esc = _lib.earlyfusion(bank, epairs, 0.1, 10)
    ev1.record()
    torch.cuda.synchronize()
    ems = ev0.elapsed_time(ev1)
    flops = 2.0 * (1000 + 1225 + 480) * NB * NB
    esc = esc.cpu().numpy().reshape(-1, 4)

    # the CPU baseline: one worker PROCESS per granted core (spawned interpreters, BLAS at one
    # thread each), one pair per task; a thread pool serialised the restatement's Python on the
    # GIL (16 threads bought ~1.5x), so processes are what the cores really give
    import tempfile
    from oracle import ef_cpu
    ncpu = 24 * nth
    sample = np.array([epairs[p * 97 % len(epairs)] for p in range(ncpu)], np.int32)
    with tempfile.TemporaryDirectory(prefix="efcpu_") as wd:
        ref, cdt = ef_cpu.run_pool({"mfccs": mf, "ssms": ss, "chromas": ch, "chroma_med": med}, NB, sample, nth, wd)
    gpu_rows = esc[[p * 97 % len(epairs) for p in range(ncpu)]]
    agree = int(np.sum(ref == gpu_rows))
    # the canonical-order C oracle (oracle/ef_oracle.cpp, golden-pinned) on the same sample: all four
    # scores must be EQUAL (the GPU's CSMs, k-smallest means and exp follow its float order)
    cbank = {"mfccs": mf, "ssms": ss, "chromas": ch, "chroma_med": med,
             "off": np.arange(NT, dtype=np.int64) * NB, "nb": np.full(NT, NB, np.int32)}
    canon = oracle.ef_batch(cbank, sample, 0.1, nthreads=nth, K=10)
    canon_eq = int(np.sum(canon == gpu_rows))
    res["earlyfusion"] = {"metric": "song-pairs/s (EarlyFusion: 3 CSMs + kNN + WCSM fusion + 4 SW, 446 blocks)",
                          "value": round(len(epairs) / (ems * 1e-3), 1), "ms": round(ems, 3),
                          "pairs": int(len(epairs)), "dtype": "f32",
                          "roofline": {"bound": "mfma",
                                       "achieved": round(flops * len(epairs) / (ems * 1e-3) / 1e12, 3),
                                       "peak": PEAK_F32_TFLOPS, "unit": "TFLOP/s",
                                       "frac": round(flops * len(epairs) / (ems * 1e-3) / 1e12 / PEAK_F32_TFLOPS, 4),
                                       "flops_per_pair": flops},
                          "cpu_baseline": {"value": round(ncpu / cdt, 3), "cores": nth, "kind": "port",
                                           "per_process": round(ncpu / cdt / nth, 3),
                                           "sample": "%d pairs, numpy restatement + C SW oracle on %d worker "
                                                     "processes (BLAS 1 thread each), %.1f s" % (ncpu, nth, cdt)},
                          "scores_equal_to_oracle": "%d of %d" % (agree, 4 * ncpu),
                          "scores_equal_to_canonical_oracle": "%d of %d" % (canon_eq, 4 * ncpu),
                          "scores_note": "scores_equal_to_oracle: the numpy restatement (BLAS-order CSMs, the "
                                         "reference's own arithmetic), where a kNN tie can flip on random features; "
                                         "scores_equal_to_canonical_oracle: all four scores against "
                                         "oracle/ef_oracle.cpp, the same float order as the GPU (CSMs, ascending "
                                         "k-smallest means, canon_expf), pinned against the reference's golden "
                                         "CSM/OTI/binarisation/getWCSM vectors (tests/test_ef_oracle.py)"}
    # ---- SNF cross-diffusion step (f2) at Da-TACOS size
    res["snf"] = snf_path(seed)
    # ---- config 3's shape: one GPU's stripe of the 8-GPU Da-TACOS Serra09 job
    log("Da-TACOS stripe (config 3, rank 0 of 8)")
    res["datacos_stripe"] = datacos_stripe(nth, seed)
    return res


def stripe_ops(lens, r0, r1, m=9, tau=1):
    """SURVEY.md §8d ops of every unordered pair (i < j) of rows [r0, r1) for the actual track lengths:
    sum of 2*12*M_i*N_j + 32*M'_i*N'_j, split by kernel as ops_split (sweep / selects / dp)."""
    L = np.asarray(lens, np.float64)
    Lp = np.maximum(np.ceil((L - m * tau) / tau), 0)
    sufL = np.concatenate([np.cumsum(L[::-1])[::-1][1:], [0.0]])    # sum_{j > i} N_j
    sufP = np.concatenate([np.cumsum(Lp[::-1])[::-1][1:], [0.0]])   # sum_{j > i} N'_j
    gram = float(np.sum(24.0 * L[r0:r1] * sufL[r0:r1]))
    cells = float(np.sum(Lp[r0:r1] * sufP[r0:r1]))
    return {"total": gram + 32.0 * cells, "sweep": gram + 11.0 * cells, "selects": 7.0 * cells, "dp": 14.0 * cells,
            "cells": cells}


def datacos_stripe(nth, seed, world=8, rank=0, chunk=1 << 20, sample=2000):
    """Config 3's per-GPU share (BASELINE.json configs[2]: Da-TACOS Serra09 Qmax, pair matrix tiled
    across 8 GPUs) measured on this one GPU: a Da-TACOS-shaped corpus (15,000 songs, 1000 cliques x 13
    + 2000 singletons, synthetic HPCP of 350..700 frames, the hard corpus of tools/datacos_plugin.py),
    the cost-balanced row stripe rank `rank` of `world` scores (acoss.distributed.stripe_bounds, as
    all_pairwise does), in 1 M-pair acoss_crp_align calls scattered into a device stripe (the timed
    region, HIP events on the launch stream). Roofline: SURVEY §8d ops for the stripe's actual
    lengths; the one-stream kernel split of the first chunk; a sampled == check against the oracle."""
    import torch
    import oracle
    from acoss import _lib, distributed, synthetic
    from acoss.engine import ChromaBank
    t0 = time.perf_counter()
    tracks, _ = synthetic.make_hard_corpus("datacos", frames=500, seed=seed, fixed_length=False)
    T = len(tracks)
    lens = np.array([len(t) for t in tracks], np.int32)
    bounds = distributed.stripe_bounds(lens, world, symmetric=True)
    r0, r1 = bounds[rank]
    bank = ChromaBank(tracks)
    chunks = list(distributed.stripe_pair_chunks(T, r0, r1, True, chunk))
    n_pairs = int(sum(len(c) for c in chunks))
    gen_s = time.perf_counter() - t0
    blk = torch.zeros((r1 - r0, T), dtype=torch.float32, device="cuda")
    bank.crp_align(chunks[0][:8192], qmax=True)  # workspaces sized once, as all_pairwise's first chunk
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(s)
    for c in chunks:
        q = bank.crp_align(c, qmax=True)["qmax"]
        p = torch.as_tensor(c.astype(np.int64)).cuda()
        blk[p[:, 0] - r0, p[:, 1]] = q
    ev1.record(s)
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1)
    ops = stripe_ops(lens, r0, r1)
    rate = n_pairs / (ms * 1e-3)
    achieved = ops["total"] / (ms * 1e-3) / 1e12
    # the first chunk on ONE stream with the library's per-phase events: the kernel split
    first = chunks[0]
    fr0, fr1 = int(first[0, 0]), int(first[-1, 0]) + 1
    prev = os.environ.get("ACOSS_SPLIT_STREAMS")
    os.environ["ACOSS_SPLIT_STREAMS"] = "1"
    _lib.profile_enable(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    bank.crp_align(first, qmax=True)
    e1.record(s)
    torch.cuda.synchronize()
    one_ms = e0.elapsed_time(e1)
    phases = _lib.profile_read()
    _lib.profile_enable(False)
    if prev is None:
        del os.environ["ACOSS_SPLIT_STREAMS"]
    else:
        os.environ["ACOSS_SPLIT_STREAMS"] = prev
    # ops of exactly the first chunk's pairs (its last row may be cut by the chunk boundary)
    fi, fj = first[:, 0], first[:, 1]
    Lf = lens.astype(np.float64)
    Lpf = np.maximum(Lf - 9, 0)
    fcells = float(np.sum(Lpf[fi] * Lpf[fj]))
    fsplit = {"sweep": float(np.sum(24.0 * Lf[fi] * Lf[fj])) + 11.0 * fcells, "selects": 7.0 * fcells,
              "dp": 14.0 * fcells}
    kernels = {}
    for k, v in phases.items():
        kops = PHASE_OPS[k](fsplit) if k in PHASE_OPS else 0.0
        kernels[k] = {"ms": round(v[0], 3), "launches": v[1],
                      "frac": round(kops / (v[0] * 1e-3) / 1e12 / PEAK_F32_TFLOPS, 4) if kops and v[0] > 0 else None}
    # sampled pairs of the stripe against the oracle (bit for bit)
    from acoss.synthetic import pack
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    allp = np.concatenate(chunks)
    sp = allp[np.sort(rng.choice(len(allp), size=min(sample, len(allp)), replace=False))]
    feats, off, ln = pack(tracks)
    tq = time.perf_counter()
    oq, _, _ = oracle.crp_batch(feats, off, ln, sp, dmax=False, nthreads=nth)
    odt = time.perf_counter() - tq
    gq = blk[torch.as_tensor(sp[:, 0] - r0).long().cuda(), torch.as_tensor(sp[:, 1]).long().cuda()].cpu().numpy()
    job = T * (T - 1) // 2
    del blk, bank
    torch.cuda.empty_cache()
    return {"metric": "song-pairs/s (Serra09 CRP+Qmax, Da-TACOS shape, rank %d of a %d-GPU stripe split)" % (rank, world),
            "value": round(rate, 1), "ms": round(ms, 3), "pairs": n_pairs, "dtype": "f32",
            "config": "Da-TACOS benchmark shape: %d songs (1000 x 13 + 2000 singletons), hard synthetic HPCP of "
                      "%d..%d frames (mean %.0f), stripe rows [%d, %d) of %d, %d acoss_crp_align calls of <= %d "
                      "pairs, scattered into a device stripe" % (T, lens.min(), lens.max(), lens.mean(), r0, r1, T,
                                                                  len(chunks), chunk),
            "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_F32_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_F32_TFLOPS, 4), "ops": ops["total"],
                         "ops_per_pair_mean": round(ops["total"] / n_pairs, 1),
                         "one_stream_first_chunk": {"pairs": int(len(first)), "rows": [fr0, fr1], "ms": round(one_ms, 3),
                                                    "kernels": kernels}},
            "projected_job_s_on_%d_gpus" % world: round(job / world / rate, 1),
            "oracle_sample": {"pairs": int(len(sp)), "qmax_equal": int(np.sum(gq == oq)),
                              "bitexact": bool(np.array_equal(gq, oq)), "oracle_s": round(odt, 2), "threads": nth},
            "setup_s": round(gen_s, 1)}


def snf_path(seed, n=15000, L=2, K=20):
    """One SNF cross-diffusion step (acoss_snf_step, similarity_fusion.py:163-174) on n x n float64
    matrices, n = 15,000 (Da-TACOS), L = 2 (ChenFusion), K = 20; HBM-bound: algorithmic bytes
    (L + 4) * 8 n^2 per step. The CPU baseline is the reference's own scipy
    expression (np_oracle.snf_step; scipy's sparse products are single-threaded, so one core) on
    the SAME inputs at the same n, and the GPU step is checked against it bit for bit."""
    import torch
    from acoss import _lib
    from oracle import np_oracle as npo
    rng = np.random.Generator(np.random.PCG64(seed))
    cm = [rng.random((n, n)) for _ in range(L)]
    cJ = np.stack([rng.choice(n, K, replace=False) for _ in range(n)]).astype(np.int32)
    cV = rng.random((n, K))
    cV /= cV.sum(1, keepdims=True)
    mats = [torch.as_tensor(m).cuda() for m in cm]
    J = torch.as_tensor(cJ).cuda()
    V = torch.as_tensor(cV).cuda()
    out = torch.empty((n, n), dtype=torch.float64, device="cuda")
    _lib.snf_step(mats, 0, J, V, 1.0, out=out)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for r in range(5):
        ev0.record(s)
        _lib.snf_step(mats, 0, J, V, 1.0, out=out, validated=True)
        ev1.record(s)
        ev1.synchronize()
        ts.append(ev0.elapsed_time(ev1))
    ms = float(np.median(ts))
    got = out.cpu().numpy()
    del mats, out
    torch.cuda.empty_cache()
    algo = (L + 4) * 8.0 * n * n
    t0 = time.perf_counter()
    ref = npo.snf_step(cm, 0, cJ, cV, 1.0)
    cdt = time.perf_counter() - t0
    same = bool(np.array_equal(got, ref))
    del ref, got, cm
    return {"metric": "SNF cross-diffusion steps/s (n = %d, L = %d, K = %d)" % (n, L, K),
            "value": round(1e3 / ms, 2), "ms": round(ms, 3), "dtype": "f64",
            "roofline": {"bound": "hbm", "achieved": round(algo / (ms * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": round(algo / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                         "bytes_per_step": algo},
            "cpu_baseline": {"value": round(1.0 / cdt, 4), "cores": 1, "kind": "port",
                             "sample": "one step at the same n = %d on the same inputs (scipy csr, "
                                       "np_oracle.snf_step, single-threaded), %.1f s" % (n, cdt)},
            "bitexact_vs_scipy": same}


def exchange_diagnostics(world, rank, comp_ms, exch_ms, probe_ms, bounds, lens, n_tracks, device):
    """Per-rank view of one multi-GPU step, assembled on rank 0 (None elsewhere):
    every rank's compute ms per step (HIP events around crp_align + the stripe scatter), exchange ms
    per step (around the stripe all-gather, so it includes waiting for the slowest rank), its
    stripe's share of the sum of M'*N' over all pairs, the max/min imbalance of both, and the
    all-gather's achieved bandwidth from a probe run after a barrier (no straggler wait inside).
    One all-gather of a 5-float row per rank (a device tensor under nccl, host under gloo)."""
    import torch
    import torch.distributed as dist
    from acoss import distributed
    costs = distributed.row_costs(lens, symmetric=True)
    r0, r1 = bounds[rank]
    mine = torch.tensor([comp_ms, exch_ms, probe_ms, float(costs[r0:r1].sum()),
                         float(sum(n_tracks - i - 1 for i in range(r0, r1)))], dtype=torch.float64, device=device)
    rows = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(rows, mine)
    if rank != 0:
        return None
    rows = [r.cpu().numpy() for r in rows]
    tot = float(costs.sum())
    rmax = max(b1 - b0 for b0, b1 in bounds)
    # every rank receives the other ranks' padded stripes (rmax x n float32 each)
    recv = float((world - 1) * rmax * n_tracks * 4)
    useful = float(sum((b1 - b0) for b0, b1 in bounds) * n_tracks * 4) * (world - 1) / world
    per = [{"rank": r, "rows": list(bounds[r]), "pairs": int(v[4]), "cost_share": round(v[3] / tot, 5),
            "compute_ms_per_step": round(float(v[0]), 3), "exchange_ms_per_step": round(float(v[1]), 3),
            "allgather_probe_ms": round(float(v[2]), 3)} for r, v in enumerate(rows)]
    comp = [float(v[0]) for v in rows]
    cost = [float(v[3]) for v in rows]
    probe = max(float(v[2]) for v in rows)
    return {"per_rank": per,
            "imbalance": {"compute_max_over_min": round(max(comp) / max(min(comp), 1e-9), 4),
                          "cost_max_over_min": round(max(cost) / max(min(cost), 1e-9), 4),
                          "compute_max_ms": round(max(comp), 3), "compute_min_ms": round(min(comp), 3)},
            "allgather": {"padded_rows": int(rmax), "bytes_received_per_rank": recv,
                          "probe_ms_max_over_ranks": round(probe, 3),
                          "gbps_per_rank": round(recv / (probe * 1e-3) / 1e9, 2) if probe > 0 else None,
                          "useful_gbps_per_rank": round(useful / (probe * 1e-3) / 1e9, 2) if probe > 0 else None,
                          "note": "bytes a rank receives in one all-gather of padded stripes; probe = one "
                                  "all-gather after a barrier, max over ranks"}}


def host_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota, qsrc = cgroup_cpu_quota()
    return {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cpu_model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cgroup_cpu_quota": quota,
            "cgroup_quota_file": qsrc}


def corpus_tracks(n_gpus, frames, seed, kind="hard"):
    from acoss import synthetic
    if kind == "hard" and n_gpus == 1:
        return synthetic.make_hard_corpus("covers80", frames=frames, seed=seed)
    sizes = synthetic.clique_sizes("covers80")
    target = int(round(164 * math.sqrt(n_gpus)))
    pattern = []
    while sum(pattern) < target:
        pattern.extend(sizes)
    # trim the pattern to exactly `target` tracks
    out, tot = [], 0
    for s in pattern:
        if tot >= target:
            break
        s = min(s, target - tot)
        out.append(s)
        tot += s
    if kind == "hard":  # the covers80 pattern repeated to the weak-scaling corpus size
        tracks, labels = [], []
        rep = 0
        while len(tracks) < target:
            tr, lab = synthetic.make_hard_corpus("covers80", frames=frames, seed=seed + rep)
            tracks += tr
            labels += [int(v) + 80 * rep for v in lab]
            rep += 1
        return tracks[:target], np.asarray(labels[:target], np.int32)
    rng = np.random.Generator(np.random.PCG64(seed))
    tracks, labels = [], []
    for lab, size in enumerate(out):
        base = synthetic.base_sequence(rng, frames)
        for v in range(size):
            seq = base if v == 0 else synthetic.cover_of(rng, base, frames)
            tracks.append(synthetic.render(rng, seq))
            labels.append(lab)
    return tracks, np.asarray(labels, np.int32)


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, script=None, argv=None):
    """`bench.py --gpus N` run without a launcher (no WORLD_SIZE in the environment): start N
    rank processes of this same command line, one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT set, as torch.distributed.run would. This parent never
    touches the GPU. Rank 0's stdout (the JSON line) is relayed; every rank's stderr passes
    through. If any rank fails the others are stopped and the exit status is non-zero."""
    import subprocess
    import tempfile
    port = _free_port()
    out0 = tempfile.TemporaryFile(mode="w+")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ACOSS_BENCH_LAUNCHER="self")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        cmd = [sys.executable, script or os.path.abspath(__file__)] + list(sys.argv[1:] if argv is None else argv)
        procs.append(subprocess.Popen(cmd, env=env,
                                      stdout=out0 if r == 0 else subprocess.DEVNULL))
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0]
            log("a rank exited with status %d: stopping the others" % rc)
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(0.2)
    out0.seek(0)
    # rank 0's JSON line only: the process group's own chatter (gloo prints its connection
    # message to stdout) goes to stderr
    for line in out0.read().splitlines():
        if line.startswith("{") and line.rstrip().endswith("}"):
            sys.stdout.write(line + "\n")
        elif line.strip():
            sys.stderr.write(line + "\n")
    sys.stdout.flush()
    return rc if rc > 0 else (1 if rc else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--frames", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=20250101)
    ap.add_argument("--corpus", choices=["hard", "bench"], default="hard")
    ap.add_argument("--cpu-sample", type=int, default=4000,
                    help="pairs timed on the CPU baseline (~15 s on the box's 16 threads at 2000 frames): "
                         "0 = skip, -1 = the whole step")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = the box's CPU share (OMP_NUM_THREADS, else every CPU this process may run on)")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-paths", action="store_true", help="skip the SiMPle / EarlyFusion lines")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return launch_ranks(args.gpus)  # before anything touches the GPU
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d: launch one rank per GPU with "
                         "--nproc-per-node equal to --gpus (or run without a launcher and let bench.py start "
                         "the ranks)" % (args.gpus, world))

    import torch
    import torch.distributed as dist
    from acoss import _lib, distributed, evaluation
    from acoss.engine import ChromaBank

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU over RCCL ("nccl"); ACOSS_DIST_BACKEND=gloo rehearses the multi-rank
    # path with several ranks sharing one GPU (the stripes are exchanged through host memory)
    backend = os.environ.get("ACOSS_DIST_BACKEND", "nccl")
    n_dev = torch.cuda.device_count()
    if world > 1 and backend == "nccl" and n_dev < world:
        raise SystemExit("bench.py: %d ranks over RCCL need %d GPUs, %d visible (ACOSS_DIST_BACKEND=gloo "
                         "rehearses several ranks on one GPU)" % (world, world, n_dev))
    dev = local % max(1, n_dev)
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    n_gpus = world

    tracks, labels = corpus_tracks(n_gpus, args.frames, args.seed, args.corpus)
    log("corpus: %d tracks x %d frames (%s)" % (len(tracks), args.frames, args.corpus))
    T = len(tracks)
    lens = np.array([len(t) for t in tracks], np.int32)
    bank = ChromaBank(tracks)
    bounds = distributed.stripe_bounds(lens, world, symmetric=True)
    r0, r1 = bounds[rank]
    my_pairs_np = distributed.stripe_pairs(T, r0, r1, symmetric=True)
    my_pairs = torch.as_tensor(my_pairs_np).cuda()
    total_pairs = T * (T - 1) // 2

    # at N > 1 every timed step also records HIP events around its compute and its exchange on the
    # stream they run on (no synchronisation inside the timed region), for the per-rank diagnostics
    step_events = []

    def step(timed=False):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if timed and world > 1 else None
        if evs:
            evs[0].record()
        out = bank.crp_align(my_pairs, qmax=True)
        blk = distributed.scatter_stripe(my_pairs, out["qmax"], r0, r1, T)
        if world > 1:
            if evs:
                evs[1].record()
            full = distributed.all_gather_stripes(blk, bounds)
            if evs:
                evs[2].record()
                step_events.append(evs)
            return full
        return blk

    def barrier():
        if world > 1:
            dist.barrier()

    log("warmup")
    for _ in range(args.warmup):
        D = step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        D = step(timed=True)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    multi = None
    if world > 1:
        comp_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in step_events]))
        exch_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in step_events]))
        blk = distributed.scatter_stripe(my_pairs, bank.crp_align(my_pairs, qmax=True)["qmax"], r0, r1, T)
        probes = []
        for _ in range(3):  # the all-gather alone: after a barrier, so no rank waits for a straggler
            torch.cuda.synchronize()
            barrier()
            pe0, pe1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            pe0.record()
            distributed.all_gather_stripes(blk, bounds)
            pe1.record()
            torch.cuda.synchronize()
            probes.append(pe0.elapsed_time(pe1))
        multi = exchange_diagnostics(world, rank, comp_ms, exch_ms, float(np.median(probes)), bounds, lens, T,
                                     "cuda" if backend == "nccl" else "cpu")
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt / args.steps * 1e3
    value = total_pairs * args.steps / dt

    # ---- one call of the path timed with HIP events on the stream it is launched on ----
    # (a) as the timed steps run it (two streams: one sub-batch's selects overlap the next one's
    #     sweep) -> roofline.achieved; (b) with ACOSS_SPLIT_STREAMS=1 and the library's per-phase
    #     events, so the kernel durations add up to that call's time -> roofline.kernels
    phases = {}
    call_ms = call1_ms = None
    if not args.no_profile:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        bank.crp_align(my_pairs, qmax=True)
        ev1.record()
        torch.cuda.synchronize()
        call_ms = ev0.elapsed_time(ev1)
        prev = os.environ.get("ACOSS_SPLIT_STREAMS")
        os.environ["ACOSS_SPLIT_STREAMS"] = "1"
        _lib.profile_enable(True)
        ev0.record()
        bank.crp_align(my_pairs, qmax=True)
        ev1.record()
        torch.cuda.synchronize()
        call1_ms = ev0.elapsed_time(ev1)
        phases = _lib.profile_read()
        _lib.profile_enable(False)
        if prev is None:
            del os.environ["ACOSS_SPLIT_STREAMS"]
        else:
            os.environ["ACOSS_SPLIT_STREAMS"] = prev

    # ---- MAP / MR1 on the assembled matrix (reference normalisation + evaluation) ----
    Dfull = D.cpu().numpy()                                       # (T, T) upper triangle filled
    Dsym = (Dfull + Dfull.T).astype(np.float32)                    # all_pairwise: Ds += Ds.T (:188-191)
    Dsym = (Dsym / np.sqrt(lens.astype(np.float64))[None, :]).astype(np.float32)  # normalize_by_length (:71-83)
    MR, MRR, MDR, MAP, tops = evaluation.eval_statistics(Dsym, labels)

    result = None
    if rank == 0:
        M = N = args.frames
        opp = ops_pair(M, N)
        split = ops_split(M, N)
        launch_ms = call_ms if call_ms else ms_per_step
        batch_pairs = len(my_pairs_np)
        kernels = {}
        for k, v in phases.items():
            ops = PHASE_OPS[k](split) * batch_pairs if k in PHASE_OPS else 0.0
            kernels[k] = {"ms": round(v[0], 3), "launches": v[1],
                          "tops": round(ops / (v[0] * 1e-3) / 1e12, 3) if ops and v[0] > 0 else None,
                          "frac": round(ops / (v[0] * 1e-3) / 1e12 / PEAK_F32_TFLOPS, 4) if ops and v[0] > 0 else None}
        dom = max(kernels.items(), key=lambda kv: kv[1]["ms"])[0] if kernels else None
        achieved = opp * batch_pairs / (launch_ms * 1e-3) / 1e12
        traffic, valu, prof_build, prof_refused = None, None, None, []
        build = build_id()
        for name, key in (("traffic_latest.json", "hbm_bytes_per_launch"), ("valu_latest.json", None)):
            tfile = os.path.join(ROOT, "profiles", name)
            if not os.path.exists(tfile):
                continue
            try:  # measured by profiles/profile.sh on the same workload: only valid at that length/corpus
                tj = json.load(open(tfile))  # and only for THIS build of the kernels
                if tj.get("frames") != args.frames or tj.get("corpus", "bench") != args.corpus:
                    continue
                if (tj.get("build") or {}).get("src_sha16") != build["src_sha16"]:
                    prof_refused.append("%s: measured on build %s, this is %s" % (
                        name, (tj.get("build") or {}).get("src_sha16"), build["src_sha16"]))
                    continue
                prof_build = tj.get("build")
                if key:
                    traffic = tj.get(key)
                else:
                    valu = tj
            except Exception:
                pass
        kernel_ms_sum = sum(v[0] for v in phases.values()) if phases else None
        roofline = {"bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_F32_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / PEAK_F32_TFLOPS, 4), "traffic": traffic,
                    "kernel": "acoss_crp_align (one call = oti + sweep/select_rows + select_cols + dp_qmax on "
                              "%d pairs; key-plane sub-batches on two streams)" % batch_pairs,
                    "ops_per_pair": opp, "ops_split_per_pair": split, "launch_ms": round(launch_ms, 3),
                    "one_stream_call_ms": round(call1_ms, 3) if call1_ms else None,
                    "kernel_ms_sum_one_stream": round(kernel_ms_sum, 3) if kernel_ms_sum else None,
                    "dominant_kernel": dom, "kernels": kernels,
                    "valu_issue": valu,
                    # the Serra09 path issues no MFMA (its 12-deep Gram runs as packed-FP32 VALU,
                    # DESIGN.md §3); gram_frac = the §8d MFMA-shaped share (2*12*M*N flops/pair)
                    # at this rate against the fp32 matrix peak
                    "mfma_frac": 0.0,
                    "gram_frac": round(2.0 * 12 * args.frames * args.frames * batch_pairs / (launch_ms * 1e-3)
                                       / 1e12 / PEAK_F32_TFLOPS, 4),
                    "traffic_build": prof_build, "traffic_refused": prof_refused or None}
        if traffic:  # the same call against the HBM roofline of the bytes it actually moves
            bpp = traffic / batch_pairs
            bound = 8e12 / bpp
            roofline["hbm_traffic"] = {"bytes_per_pair": round(bpp), "algorithmic_bytes_per_pair": 4 * 12 * 2 * args.frames,
                                       "pairs_per_s_at_8TBps": round(bound, 1),
                                       "frac": round(batch_pairs / (launch_ms * 1e-3) / bound, 4)}

        map_parity, cpu = None, None
        if world == 1 and args.corpus == "hard":
            map_parity = oracle_map_parity(tracks, labels, lens, my_pairs_np, Dfull, Dsym, args.frames,
                                           (MR, MRR, MDR, MAP, tops))
        nth, nth_src = (args.cpu_threads, "--cpu-threads") if args.cpu_threads else cpu_share()
        if args.cpu_sample != 0 and world == 1:  # the CPU baseline: rank 0 at N = 1 only
            import oracle
            from acoss.synthetic import pack
            feats, off, ln = pack(tracks)
            rng = np.random.Generator(np.random.PCG64(1234))
            k = min(args.cpu_sample if args.cpu_sample > 0 else len(my_pairs_np), len(my_pairs_np))
            sp = my_pairs_np[np.sort(rng.choice(len(my_pairs_np), size=k, replace=False))]
            what = ("the whole step: all %d pairs" % k) if k == len(my_pairs_np) else \
                   ("%d random pairs of the step's %d" % (k, len(my_pairs_np)))
            log("cpu baseline: %s on %d threads" % (what, nth))
            t0 = time.perf_counter()
            q, _, _ = oracle.crp_batch(feats, off, ln, sp, dmax=False, nthreads=nth)
            cdt = time.perf_counter() - t0
            gq = Dfull[sp[:, 0], sp[:, 1]]
            cpu = {"value": round(len(sp) / cdt, 3), "unit": "song-pairs/s", "cores": nth, "kind": "port",
                   "per_thread": round(len(sp) / cdt / nth, 3), "threads_from": nth_src,
                   "sample": "%s (%dx%d frames), oracle/crp_oracle.cpp, %d OpenMP threads (%s), "
                             "%.1f s" % (what, args.frames, args.frames, nth, nth_src, cdt),
                   "host": host_info(),
                   "qmax_bitexact_vs_gpu": bool(np.array_equal(gq.astype(np.float32), q)),
                   "qmax_pairs_differing": int(np.sum(gq.astype(np.float32) != q))}

        paths = None
        if world == 1 and not args.no_paths:
            log("other paths (SiMPle, EarlyFusion, SNF)")
            paths = other_paths(nth, args.seed)

        result = {
            "metric": "song-pairs/sec (CSM+Qmax) on 12-d HPCP, ~2000 frames/track; MAP parity",
            "value": round(value, 2), "unit": "song-pairs/s", "n_gpus": n_gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "covers80-shaped synthetic HPCP (%s corpus), Serra09 CRP+Qmax, all unordered pairs"
                                   % args.corpus,
                       "tracks": T, "pairs_per_step": total_pairs, "frames_per_track": args.frames,
                       "m": 9, "tau": 1, "kappa": 0.095, "oti": True, "parallelism": "pair-matrix row stripes dp%d"
                       % n_gpus},
            "map": round(float(MAP), 6), "mr1": round(float(MR), 4), "mrr": round(float(MRR), 6),
            "top1": int(tops[0]), "map_parity": map_parity,
            "roofline": roofline, "cpu_baseline": cpu,
            "speedup_vs_cpu": round(value / cpu["value"], 1) if cpu else None,
            "other_paths": paths,
            "build": build,
            "launch": {"world": world, "device_count": n_dev, "backend": backend if world > 1 else None,
                       "launcher": os.environ.get("ACOSS_BENCH_LAUNCHER", "external" if world > 1 else None)},
            "multi_gpu": multi,
        }
    if world > 1 and not args.no_paths:
        # SNF late fusion at Da-TACOS size across the ranks: the measured sharding decision
        # (similarity_fusion.shard_plan: one replicated step vs one all-gather of B, max over ranks)
        log("SNF sharding plan (n = 15,000)")
        snf = snf_shard_probe(world, rank, args.seed)
        if result is not None:
            result["snf_plan"] = snf
    if result is not None:
        print(json.dumps(result))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def snf_shard_probe(world, rank, seed, n=15000, L=2, K=20):
    """similarity_fusion.shard_plan on ChenFusion-shaped inputs (L = 2 float64 n x n matrices, K = 20)
    at Da-TACOS size: times one replicated acoss_snf_step and one all-gather of B's row stripes
    (RCCL over xGMI under the nccl backend), and reports the decision the fusion would take."""
    import torch
    from acoss.algorithms.utils import similarity_fusion as sf
    g = torch.Generator(device="cuda").manual_seed(seed)
    Pts = [torch.rand((n, n), dtype=torch.float64, device="cuda", generator=g) for _ in range(L)]
    rng = np.random.Generator(np.random.PCG64(seed))
    J = torch.as_tensor(np.stack([rng.choice(n, K, replace=False) for _ in range(n)]).astype(np.int32)).cuda()
    V = torch.as_tensor(rng.random((n, K))).cuda()
    plan = sf.shard_plan(Pts, [J] * L, [V] * L, 1.0, world, rank, force=None)
    del Pts
    torch.cuda.empty_cache()
    return plan


if __name__ == "__main__":
    sys.exit(main())
