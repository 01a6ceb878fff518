"""Cover-ID evaluation statistics (MR, MRR, MDR, MAP, Top-k), vectorised.

Restates CoverAlgorithm.getEvalStatistics (acoss/algorithms/algorithm_template.py:206-291):
for every song in a clique of size >= 2, the 1-based ranks of the other clique members in
its row of D sorted by decreasing score (the song itself excluded via diag = -inf, :234);
MR/MRR/MDR use the first such rank, MAP the mean precision at each rank (:258-263);
MRR divides by ALL N songs (:267), as the reference does.

Ties: the reference's np.argsort(-D, 1) is unstable (:235), so its order among equal scores
is platform-dependent. Here ties are broken by the reference's own row reordering (cliques
contiguous, larger cliques first, :220-230) made deterministic (stable sorts, members in
ascending index). With tie-free scores the result equals the reference's exactly
(tests/test_evaluation.py pins it against golden vectors captured from the reference).
"""
import os

import numpy as np


def clique_order(labels):
    """Permutation used by the reference: cliques contiguous, biggest first."""
    labels = np.asarray(labels)
    uniq, first, inv, counts = np.unique(labels, return_index=True, return_inverse=True, return_counts=True)
    # cliques in order of first appearance (dict insertion order in the reference), then
    # stable sort by decreasing size
    by_first = np.argsort(first, kind="stable")
    order = by_first[np.argsort(-counts[by_first], kind="stable")]
    perm = np.concatenate([np.flatnonzero(inv == c) for c in order]) if len(order) else np.zeros(0, int)
    return perm, counts[order]


def eval_statistics(D, labels, topsidx=(1, 10, 100, 1000)):
    """Return (MR, MRR, MDR, MAP, tops) exactly as getEvalStatistics computes them, with the
    cliques given as one label per song (cliques ordered by first appearance)."""
    perm, Ks = clique_order(labels)
    cliques, start = [], 0
    for K in Ks:
        cliques.append(perm[start:start + K].tolist())
        start += K
    return eval_statistics_cliques(D, cliques, topsidx, presorted=True)


def eval_statistics_cliques(D, cliques, topsidx=(1, 10, 100, 1000), presorted=False):
    """getEvalStatistics on explicit cliques (lists of song indices, in the order of the
    reference's `self.cliques` dict). Cliques are stably sorted by decreasing size (:219-225)
    unless `presorted`."""
    D = np.array(D, dtype=np.float32)
    N = D.shape[0]
    Ks = np.array([len(c) for c in cliques], dtype=np.int64)
    if not presorted:
        order = np.argsort(-Ks, kind="stable")
        cliques = [cliques[i] for i in order]
        Ks = Ks[order]
    perm = np.array([i for c in cliques for i in c], dtype=np.int64)
    D = D[perm][:, perm]
    np.fill_diagonal(D, -np.inf)
    ranks = np.full(N, np.nan)
    allmap = np.full(N, np.nan)
    # row-wise descending order, stable (index order breaks ties)
    order = np.argsort(-D, axis=1, kind="stable")
    pos = np.empty_like(order)
    rows = np.arange(N)[:, None]
    pos[rows, order] = np.arange(N)[None, :]
    start = 0
    for K in Ks:
        if K < 2:
            break
        members = np.arange(start, start + K)
        for i in members:
            others = members[members != i]
            r = np.sort(pos[i, others]) + 1
            ranks[i] = r[0]
            allmap[i] = np.mean(np.arange(1, K) / r)
        start += K
    MAP = np.nanmean(allmap) if np.any(~np.isnan(allmap)) else np.nan
    ranks = ranks[~np.isnan(ranks)]
    MR = np.mean(ranks) if len(ranks) else np.nan
    MRR = 1.0 / N * np.sum(1.0 / ranks)
    MDR = np.median(ranks) if len(ranks) else np.nan
    tops = np.array([np.sum(ranks <= t) for t in topsidx], dtype=np.float64)
    return MR, MRR, MDR, MAP, tops


def write_results_csv(resultsfile, name, similarity_type, stats, topsidx=(1, 10, 100, 1000)):
    """Append one row in the reference's results CSV format (algorithm_template.py:277-290)."""
    MR, MRR, MDR, MAP, tops = stats
    new = not os.path.exists(resultsfile)
    with open(resultsfile, "a") as fout:
        if new:
            fout.write("name, MR, MRR, MDR, MAP")
            for t in topsidx:
                fout.write(",Top-%i" % t)
            fout.write("\n")
        fout.write("%s_%s," % (name, similarity_type))
        fout.write("%.3g, %.3g, %.3g, %.3g" % (MR, MRR, MDR, MAP))
        for t in tops:
            fout.write(", %.3g" % t)
        fout.write("\n")
