"""Configs 3 and 4 at full size through the reference's plugin API on ONE GPU (BASELINE.json
configs[2..3]; VERDICT r03 "next" #3).

    python tools/datacos_plugin.py --algo serra09|simple|earlyfusion [--tracks 15000] [--frames 500]
                                   [--sample 5000] [--out result.json]

Builds the Da-TACOS benchmark clique structure (acoss/data/da-tacos_benchmark_subset.csv shape:
1000 cliques x 13 + 2000 singletons = 15,000 songs) as per-song feature files in the reference's
layout (<dir>/<work_id>/<track_id>, README.md:93-114), already at the pair kernel's length (base
500 frames: a 4-minute track's HPCP after the x40 downsample; the default "hard" corpus stretches
covers 0.7-1.4x, so MAP is below 1 and a changed score can move it), and runs the reference flow
(coverid.py:57-70,124-139) on them:

  serra09: Serra09(csv, dir, downsample_fac=1) -> all_pairwise(symmetric=True) (112.5 M unordered
           pairs) -> normalize_by_length -> getEvalStatistics('main')
  simple:  Simple(csv, dir, chroma_type='crema', WIN=2, SKIP=1) -> all_pairwise(symmetric=False)
           (225.0 M ordered pairs) -> getEvalStatistics('main')

  earlyfusion (config 5, BASELINE.json configs[4]): per-song feature files with hpcp, mfcc_htk
           (43 frames shorter than the chroma, a fixed projection of it plus noise, so covers share
           MFCC structure) and madmom onsets every --beat-period frames; the reference flow of
           coverid.py:72-88: EarlyFusion(csv, dir).prepare() (beat-block features of every song on
           the GPU, cached per song) -> all_pairwise(symmetric=True) (112.5 M unordered pairs, four
           score matrices) -> do_late_fusion() (SNF over 3 and over 4 n x n matrices) ->
           getEvalStatistics on all six keys

and checks full-size properties of the result:
  * Serra09: the raw Ds (before normalisation) is symmetric with a zero diagonal, finite everywhere;
    SiMPle: finite off the diagonal;
  * a seeded sample of --sample pairs equals the CPU oracle (oracle/, test infrastructure) exactly,
    from the same inputs (Serra09: the feature files' chroma, since downsample_fac=1 is the
    identity; SiMPle: the GPU's SiMPle features, themselves checked against the numpy restatement
    on a few songs);
  * MAP / MR1 / MRR / MDR / Top-k of the device evaluation (acoss_eval_ranks) equal the host
    restatement of getEvalStatistics on the same matrix;
  * EarlyFusion: the four score matrices symmetric with a zero diagonal and finite; the sampled
    pairs' mfccs / ssms / chromas / early scores == the canonical-order CPU oracle
    (oracle/ef_oracle.cpp, pinned against the reference's golden vectors) on the GPU's block
    features, which are checked against the numpy restatement (np_oracle.ef_block_features) on a
    few songs; the early score's agreement with the reference-order numpy composition is reported;
    late / early+late finite; device == host statistics on every key.
Prints progress, per-stage wall times, peak host RSS, and one JSON line (also written to --out).
"""
import argparse
import json
import os
import resource
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "acoss-1_amd")]

import numpy as np  # noqa: E402


def log(msg, t0=[time.perf_counter()]):
    print("[datacos %.1fs] %s" % (time.perf_counter() - t0[0], msg), file=sys.stderr, flush=True)


def rss_gb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6  # KB -> GB


def corpus(n_tracks, frames, seed, kind="hard"):
    from acoss import synthetic
    if kind == "hard":  # the discriminative corpus (shared chord phrases, partial covers): MAP < 1
        tracks, labels = synthetic.make_hard_corpus("datacos", frames=frames, seed=seed, fixed_length=False)
        return tracks[:n_tracks], np.asarray(labels[:n_tracks], np.int32)
    rng = np.random.Generator(np.random.PCG64(seed))
    tracks, labels = [], []
    for lab, size in enumerate(synthetic.clique_sizes("datacos")):
        n0 = int(round(frames * rng.uniform(0.9, 1.1)))
        base = synthetic.base_sequence(rng, n0)
        for v in range(size):
            seq = base if v == 0 else synthetic.cover_of(rng, base, int(round(n0 * rng.uniform(0.9, 1.1))))
            tracks.append(synthetic.render(rng, seq))
            labels.append(lab)
        if len(tracks) >= n_tracks:
            break
    return tracks[:n_tracks], np.asarray(labels[:n_tracks], np.int32)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", choices=["serra09", "simple", "earlyfusion"], default="serra09")
    ap.add_argument("--beat-period", type=int, default=7, help="earlyfusion: chroma frames between onsets")
    ap.add_argument("--host-eval-keys", default="all",
                    help="earlyfusion: comma-separated Ds keys whose device statistics are compared with the "
                         "host restatement (11 s each at 15,000 songs), or 'all'")
    ap.add_argument("--tracks", type=int, default=15000)
    ap.add_argument("--frames", type=int, default=500)
    ap.add_argument("--sample", type=int, default=5000)
    ap.add_argument("--seed", type=int, default=20250101)
    ap.add_argument("--corpus", choices=["hard", "easy"], default="hard",
                    help="hard: synthetic.make_hard_corpus (covers 0.7-1.4x the base length); easy: +-10 %% lengths")
    ap.add_argument("--threads", type=int, default=16, help="CPU oracle threads for the sample")
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--out", default=None)
    return ap.parse_args(argv)


def run(a):
    """The whole flow for the parsed options `a`; returns the result dict (res["ok"]: every check
    passed). Also the body of tests/test_gpu_datacos_full.py, at a short frame count."""
    if a.algo == "earlyfusion":
        return run_earlyfusion(a)
    import torch
    import oracle
    from acoss import evaluation, synthetic
    from oracle import np_oracle as npo

    stages = {}
    t = time.perf_counter()
    tracks, labels = corpus(a.tracks, a.frames, a.seed, a.corpus)
    T = len(tracks)
    lens = np.array([len(x) for x in tracks], np.int32)
    work = a.workdir or tempfile.mkdtemp(prefix="datacos_")
    key = "hpcp" if a.algo == "serra09" else "crema"
    csv, fdir = synthetic.write_feature_dataset(work, tracks, labels, chroma_keys=(key,))
    stages["write_features_s"] = round(time.perf_counter() - t, 2)
    log("%d songs (%d cliques), frames %d..%d, feature files written in %.1f s" %
        (T, len(set(labels.tolist())), lens.min(), lens.max(), stages["write_features_s"]))
    cache = os.path.join(work, "cache")
    torch.cuda.set_device(0)

    t = time.perf_counter()
    if a.algo == "serra09":
        from acoss.algorithms.rqa_serra09 import Serra09
        algo = Serra09(csv, fdir, chroma_type=key, shortname="datacos", downsample_fac=1, cachedir=cache)
        symmetric = True
    else:
        from acoss.algorithms.simple_silva import Simple
        algo = Simple(csv, fdir, chroma_type=key, shortname="datacos", WIN=2, SKIP=1, cachedir=cache)
        symmetric = False
    algo.prepare()
    torch.cuda.synchronize()
    stages["prepare_s"] = round(time.perf_counter() - t, 2)
    log("prepare %.1f s" % stages["prepare_s"])

    t = time.perf_counter()
    algo.all_pairwise(symmetric=symmetric)
    torch.cuda.synchronize()
    stages["all_pairwise_s"] = round(time.perf_counter() - t, 2)
    n_pairs = T * (T - 1) // (2 if symmetric else 1)
    log("all_pairwise: %d pairs in %.1f s = %.0f pairs/s" % (n_pairs, stages["all_pairwise_s"],
                                                             n_pairs / stages["all_pairwise_s"]))

    checks = {}
    D = np.asarray(algo.Ds["main"])
    off = ~np.eye(T, dtype=bool)
    checks["finite_off_diagonal"] = bool(np.isfinite(D[off]).all())
    if symmetric:
        checks["symmetric"] = bool(np.array_equal(D, D.T))
        checks["diagonal_zero"] = bool(np.all(np.diag(D) == 0))
    rng = np.random.Generator(np.random.PCG64(a.seed + 1))
    if symmetric:
        i = rng.integers(0, T, size=4 * a.sample)
        j = rng.integers(0, T, size=4 * a.sample)
        m = i < j
        u = np.unique(np.stack([i[m], j[m]], 1), axis=0)
    else:
        i = rng.integers(0, T, size=2 * a.sample)
        j = rng.integers(0, T, size=2 * a.sample)
        m = i != j
        u = np.unique(np.stack([i[m], j[m]], 1), axis=0)
    sp = u[np.sort(rng.permutation(len(u))[:a.sample])].astype(np.int32)  # uniform over the matrix
    t = time.perf_counter()
    if a.algo == "serra09":
        feats, foff, flen = synthetic.pack(tracks)
        q, _, _ = oracle.crp_batch(feats, foff, flen, sp, dmax=False, nthreads=a.threads)
        got = D[sp[:, 0], sp[:, 1]]
        checks["feature_identity"] = bool(all(np.array_equal(algo.all_feats[k], tracks[k]) for k in range(0, T, 997)))
    else:
        feats = [algo.all_feats[k] for k in range(T)]
        for k in range(0, T, 1499):
            np.testing.assert_allclose(feats[k], npo.simple_features(tracks[k], win=2, skip=1), rtol=1e-12,
                                       atol=1e-15)
        checks["simple_features_vs_restatement_1e-12"] = True
        flat = np.concatenate([f.ravel() for f in feats])
        soff = np.concatenate([[0], np.cumsum([f.size for f in feats])[:-1]]).astype(np.int64)
        slen = np.array([f.shape[1] for f in feats], np.int32)
        cs, _ = oracle.simple_batch(flat, soff, slen, sp, nthreads=a.threads)
        q = (-cs).astype(np.float32)
        got = D[sp[:, 0], sp[:, 1]]
    checks["sample_pairs"] = int(len(sp))
    checks["sample_pairs_differing_from_oracle"] = int(np.sum(got != q))
    stages["oracle_sample_s"] = round(time.perf_counter() - t, 2)
    log("oracle sample: %d pairs, %d differ (%.1f s)" % (len(sp), checks["sample_pairs_differing_from_oracle"],
                                                         stages["oracle_sample_s"]))
    del D

    if a.algo == "serra09":
        t = time.perf_counter()
        algo.normalize_by_length()
        stages["normalize_s"] = round(time.perf_counter() - t, 2)
    t = time.perf_counter()
    MR, MRR, MDR, MAP, tops = algo.getEvalStatistics("main")
    stages["eval_device_s"] = round(time.perf_counter() - t, 2)
    t = time.perf_counter()
    cliques = [sorted(algo.cliques[s]) for s in algo.cliques]
    hMR, hMRR, hMDR, hMAP, htops = evaluation.eval_statistics_cliques(np.array(algo.Ds["main"], np.float32), cliques,
                                                                     [1, 10, 100, 1000])
    stages["eval_host_s"] = round(time.perf_counter() - t, 2)
    checks["eval_device_equals_host"] = bool(MR == hMR and MRR == hMRR and MDR == hMDR and MAP == hMAP
                                             and list(tops) == list(htops))
    ok = all(v for k, v in checks.items() if isinstance(v, bool)) and checks["sample_pairs_differing_from_oracle"] == 0
    res = {"algo": a.algo, "config": "Da-TACOS benchmark shape, %d songs (1000 x 13 + singletons), %s corpus, "
                                     "frames %d..%d (base %d)" % (T, a.corpus, lens.min(), lens.max(), a.frames),
           "api": ("Serra09(downsample_fac=1).all_pairwise(symmetric=True) -> normalize_by_length -> getEvalStatistics"
                   if a.algo == "serra09" else
                   "Simple(chroma_type='crema', WIN=2, SKIP=1).all_pairwise(symmetric=False) -> getEvalStatistics"),
           "pairs": n_pairs, "pairs_per_s_all_pairwise": round(n_pairs / stages["all_pairwise_s"], 1),
           "stages": stages, "peak_host_rss_gb": round(rss_gb(), 2),
           "MAP": float(MAP), "MR1": float(MR), "MRR": float(MRR), "MDR": float(MDR), "top": [int(x) for x in tops],
           "checks": checks, "ok": bool(ok), "gpu": torch.cuda.get_device_name(0)}
    algo.cleanup_memmap()
    if not a.workdir:
        shutil.rmtree(work, ignore_errors=True)
    return res


def _sample_pairs(rng, T, n):
    i = rng.integers(0, T, size=4 * n)
    j = rng.integers(0, T, size=4 * n)
    m = i < j
    u = np.unique(np.stack([i[m], j[m]], 1), axis=0)
    return u[np.sort(rng.permutation(len(u))[:n])].astype(np.int32)  # uniform over the upper triangle


def run_earlyfusion(a):
    """Config 5 through the reference flow (coverid.py:72-88) at the given track count."""
    import torch
    import oracle
    from acoss import evaluation, synthetic
    from acoss.algorithms.earlyfusion_traile import EarlyFusion
    from acoss.algorithms.utils import similarity_fusion as sf
    from oracle import np_oracle as npo

    stages = {}
    t = time.perf_counter()
    tracks, labels = corpus(a.tracks, a.frames, a.seed, a.corpus)
    T = len(tracks)
    lens = np.array([len(x) for x in tracks], np.int32)
    work = a.workdir or tempfile.mkdtemp(prefix="datacos_ef_")
    csv, fdir = synthetic.write_feature_dataset(work, tracks, labels, with_mfcc=True, beat_period=a.beat_period,
                                                chroma_keys=("hpcp",), mfcc_from_chroma=True)
    stages["write_features_s"] = round(time.perf_counter() - t, 2)
    log("%d songs (%d cliques), chroma frames %d..%d, onsets every ~%d frames, files written in %.1f s" %
        (T, len(set(labels.tolist())), lens.min(), lens.max(), a.beat_period, stages["write_features_s"]))
    cache = os.path.join(work, "cache")
    torch.cuda.set_device(0)

    t = time.perf_counter()
    algo = EarlyFusion(csv, fdir, chroma_type="hpcp", shortname="datacos", cachedir=cache)
    algo.prepare()  # coverid.py:80-81's load_features loop, batched
    torch.cuda.synchronize()
    stages["prepare_s"] = round(time.perf_counter() - t, 2)
    nb = algo.track_lengths()
    log("prepare %.1f s: beat blocks per song %d..%d (mean %.1f)" % (stages["prepare_s"], nb.min(), nb.max(),
                                                                     nb.mean()))

    t = time.perf_counter()
    algo.all_pairwise(symmetric=True)
    torch.cuda.synchronize()
    stages["all_pairwise_s"] = round(time.perf_counter() - t, 2)
    n_pairs = T * (T - 1) // 2
    log("all_pairwise: %d pairs in %.1f s = %.0f pairs/s" % (n_pairs, stages["all_pairwise_s"],
                                                             n_pairs / stages["all_pairwise_s"]))
    checks = {}
    keys4 = ("mfccs", "ssms", "chromas", "early")
    for k in keys4:
        D = np.asarray(algo.Ds[k])
        checks["%s_finite" % k] = bool(np.isfinite(D).all())
        checks["%s_symmetric" % k] = bool(np.array_equal(D, D.T))
        checks["%s_diagonal_zero" % k] = bool(np.all(np.diag(D) == 0))
        del D

    # block features of a few songs against the numpy restatement (float32 roundings apart)
    t = time.perf_counter()
    from acoss.features_io import load_features
    close = True
    for k in range(0, T, max(1, T // 6)):
        f = load_features(algo.filepaths[k])
        ref = npo.ef_block_features(f["hpcp"], f["mfcc_htk"], f["madmom_features"]["onsets"])
        for key in ("mfccs", "ssms", "chromas"):
            g = algo.all_block_feats[k][key]
            close &= g.shape == ref[key].shape and bool(np.allclose(g, ref[key], rtol=1e-5, atol=2e-6))
    checks["block_features_vs_restatement_1e-5"] = bool(close)
    stages["block_check_s"] = round(time.perf_counter() - t, 2)

    # sampled pairs against the canonical-order oracle on the GPU's block features
    t = time.perf_counter()
    rng = np.random.Generator(np.random.PCG64(a.seed + 1))
    sp = _sample_pairs(rng, T, a.sample)
    feats = [algo.all_block_feats[k] for k in range(T)]
    bank = {k: np.concatenate([f[k] for f in feats]) for k in ("mfccs", "ssms", "chromas")}
    bank["chroma_med"] = np.stack([np.asarray(f["chroma_med"], np.float32) for f in feats])
    bank["nb"] = nb.astype(np.int32)
    bank["off"] = np.concatenate([[0], np.cumsum(nb[:-1])]).astype(np.int64)
    ref = oracle.ef_batch(bank, sp, algo.kappa, nthreads=a.threads, K=algo.K)
    diff = {}
    for f, k in enumerate(("mfccs", "ssms", "chromas", "early")):
        got = np.asarray(algo.Ds[k])[sp[:, 0], sp[:, 1]]
        diff[k] = int(np.sum(got != ref[:, f].astype(np.float32)))
    checks["sample_pairs"] = int(len(sp))
    checks["sample_pairs_differing_from_oracle"] = int(sum(diff.values()))
    checks["sample_differing_by_key"] = diff
    # the early score is in the canonical comparison above (all 4 scores, every sampled pair); the
    # reference-order numpy composition (BLAS-order CSMs, np.partition means, numpy exp): reported
    ne = min(300, len(sp))
    early_eq = 0
    for (i, j) in sp[:ne]:
        f1, f2 = feats[i], feats[j]
        C = [npo.get_csm(f1["mfccs"], f2["mfccs"]), npo.get_csm(f1["ssms"], f2["ssms"]),
             npo.get_csm_blocked_oti(f1["chromas"], f2["chromas"], f1["chroma_med"], f2["chroma_med"],
                                     npo.get_csm_cosine)]
        W = np.zeros_like(C[0])
        for c in C:
            W += npo.getWCSM(c, algo.K, algo.K)
        e = oracle.sw_constrained(npo.csm_to_binary(np.exp(-W), algo.kappa))
        early_eq += int(np.float32(e) == algo.Ds["early"][i, j])
    checks["early_equal_to_numpy_composition"] = "%d of %d" % (early_eq, ne)
    stages["oracle_sample_s"] = round(time.perf_counter() - t, 2)
    log("oracle sample: %d pairs, differing %s; early %s (%.1f s)" % (len(sp), diff, checks[
        "early_equal_to_numpy_composition"], stages["oracle_sample_s"]))
    del bank, feats

    t = time.perf_counter()
    algo.do_late_fusion()
    torch.cuda.synchronize()
    stages["late_fusion_s"] = round(time.perf_counter() - t, 2)
    log("do_late_fusion (SNF over 3 and 4 matrices, n = %d) %.1f s" % (T, stages["late_fusion_s"]))
    for k in ("late", "early+late"):
        checks["%s_finite" % k] = bool(np.isfinite(np.asarray(algo.Ds[k])).all())

    keys = list(algo.Ds.keys())
    host_keys = keys if a.host_eval_keys == "all" else [k for k in a.host_eval_keys.split(",") if k]
    stats, t_dev, t_host = {}, 0.0, 0.0
    cliques = [sorted(algo.cliques[s]) for s in algo.cliques]
    for k in keys:
        t = time.perf_counter()
        MR, MRR, MDR, MAP, tops = algo.getEvalStatistics(k)
        t_dev += time.perf_counter() - t
        stats[k] = {"MAP": float(MAP), "MR1": float(MR), "MRR": float(MRR), "MDR": float(MDR),
                    "top": [int(x) for x in tops]}
        if k in host_keys:
            t = time.perf_counter()
            h = evaluation.eval_statistics_cliques(np.array(algo.Ds[k], np.float32), cliques, [1, 10, 100, 1000])
            t_host += time.perf_counter() - t
            checks["eval_device_equals_host_%s" % k] = bool(MR == h[0] and MRR == h[1] and MDR == h[2]
                                                            and MAP == h[3] and list(tops) == list(h[4]))
    stages["eval_device_s"] = round(t_dev, 2)
    stages["eval_host_s"] = round(t_host, 2)
    ok = all(v for v in checks.values() if isinstance(v, bool)) and checks["sample_pairs_differing_from_oracle"] == 0
    res = {"algo": "earlyfusion",
           "config": "Da-TACOS benchmark shape, %d songs (1000 x 13 + singletons), %s corpus, chroma frames "
                     "%d..%d (base %d), onsets every ~%d frames: %d..%d beat blocks per song" %
                     (T, a.corpus, lens.min(), lens.max(), a.frames, a.beat_period, nb.min(), nb.max()),
           "api": "EarlyFusion(csv, dir).prepare() -> all_pairwise(symmetric=True) -> do_late_fusion() -> "
                  "getEvalStatistics on every key (coverid.py:72-88)",
           "pairs": n_pairs, "pairs_per_s_all_pairwise": round(n_pairs / stages["all_pairwise_s"], 1),
           "mean_blocks": round(float(nb.mean()), 2), "stages": stages, "peak_host_rss_gb": round(rss_gb(), 2),
           "stats": stats, "snf_plan": dict(sf.LAST_PLAN), "checks": checks, "ok": bool(ok),
           "gpu": torch.cuda.get_device_name(0)}
    res["MAP"] = stats["early+late"]["MAP"]
    algo.cleanup_memmap()
    if not a.workdir:
        shutil.rmtree(work, ignore_errors=True)
    return res


def main():
    a = parse_args()
    res = run(a)
    ok = res["ok"]
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
