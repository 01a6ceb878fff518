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
(tests/test_host.py::test_eval_statistics_golden pins it against golden vectors captured from
the reference).
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


def _ordered_cliques(cliques, presorted):
    Ks = np.array([len(c) for c in cliques], dtype=np.int64)
    if not presorted:
        order = np.argsort(-Ks, kind="stable")
        cliques = [cliques[i] for i in order]
        Ks = Ks[order]
    perm = np.array([i for c in cliques for i in c], dtype=np.int64)
    return perm, Ks


def _stats_from_ranks(member_ranks, Ks, N, topsidx):
    """member_ranks(start, K, i) -> the 1-based ranks of the other members of the clique at
    permuted positions [start, start + K) in the row of member i (permuted position)."""
    ranks = np.full(N, np.nan)
    allmap = np.full(N, np.nan)
    start = 0
    for K in Ks:
        if K < 2:
            break
        for i in range(start, start + K):
            r = np.sort(member_ranks(start, K, i))
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


def eval_statistics_cliques(D, cliques, topsidx=(1, 10, 100, 1000), presorted=False):
    """getEvalStatistics on explicit cliques (lists of song indices, in the order of the
    reference's `self.cliques` dict). Cliques are stably sorted by decreasing size (:219-225)
    unless `presorted`."""
    D = np.array(D, dtype=np.float32)
    N = D.shape[0]
    perm, Ks = _ordered_cliques(cliques, presorted)
    D = D[perm][:, perm]
    np.fill_diagonal(D, -np.inf)
    # row-wise descending order, stable (index order breaks ties)
    order = np.argsort(-D, axis=1, kind="stable")
    pos = np.empty_like(order)
    rows = np.arange(N)[:, None]
    pos[rows, order] = np.arange(N)[None, :]

    def member_ranks(start, K, i):
        members = np.arange(start, start + K)
        return pos[i, members[members != i]] + 1
    return _stats_from_ranks(member_ranks, Ks, N, topsidx)


def eval_statistics_device(D, labels=None, cliques=None, topsidx=(1, 10, 100, 1000)):
    """eval_statistics / eval_statistics_cliques on a device-resident (N, N) float32 torch
    matrix: the O(N^2) rank step runs as one HIP kernel (acoss_eval_ranks: the clique members'
    positions in each query row's stable descending order, no sort materialised); the O(N)
    statistics are the same host code as above, so the result is identical to the host path."""
    from . import _lib
    if cliques is None:
        perm, Ks = clique_order(labels)
        perm = perm.astype(np.int64)
        Ks = np.asarray(Ks, np.int64)
    else:
        perm, Ks = _ordered_cliques(cliques, False)
    N = int(D.shape[0])
    pos = np.empty(N, np.int32)
    pos[perm] = np.arange(N, dtype=np.int32)
    q_song, m_off, members, where = [], [0], [], {}
    start = 0
    for K in Ks:
        if K < 2:
            break
        for i in range(start, start + K):
            where[i] = len(q_song)
            q_song.append(perm[i])
            others = [perm[t] for t in range(start, start + K) if t != i]
            members.extend(others)
            m_off.append(len(members))
        start += K
    if q_song:
        r = _lib.eval_ranks(D, pos, np.asarray(q_song, np.int32), np.asarray(m_off, np.int64),
                            np.asarray(members, np.int32)).astype(np.int64)
    else:
        r = np.zeros(0, np.int64)

    def member_ranks(start, K, i):
        q = where[i]
        return r[m_off[q]:m_off[q + 1]]
    return _stats_from_ranks(member_ranks, Ks, N, topsidx)


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
