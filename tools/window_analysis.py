"""Per-line threshold-window analysis behind DESIGN.md §8 item 1 (CPU only, oracle keys).

How far is each line's 9.5th-percentile squared-distance key from an estimate taken on 32
sampled cells of the line (four runs of 8 consecutive rows for a column, of 8 columns for a
row)? Narrow per-line codes in the key planes would need the true threshold inside a window
around that estimate; the fraction of lines outside [-0.75, +1.25] and [-0.5, +0.5] binades is
the fraction that would fall back to a full recompute.

    python tools/window_analysis.py [--pairs 30]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "acoss-1_amd")]

import oracle  # noqa: E402
from bench import corpus_tracks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=30)
    a = ap.parse_args()
    tracks, _ = corpus_tracks(1, 2000, 20250101)
    rng = np.random.default_rng(0)
    runs = (0.1, 0.35, 0.6, 0.85)
    cols_err, rows_err = [], []
    for _ in range(a.pairs):
        i, j = rng.choice(len(tracks), 2, replace=False)
        X, Y = np.asarray(tracks[i], np.float32), np.asarray(tracks[j], np.float32)
        K = oracle.crp_dist(X, Y, oracle.oti(oracle.profile(X), oracle.profile(Y))) ** 2
        M, N = K.shape
        true_c = np.sort(K, axis=0)[int(np.floor((M - 1) * 0.095))]
        rows = np.concatenate([np.arange(int(M * f), int(M * f) + 8) for f in runs])
        est_c = np.sort(K[rows], axis=0)[2]
        cols_err.append(np.log2(np.maximum(true_c, 1e-30) / np.maximum(est_c, 1e-30)))
        true_r = np.sort(K, axis=1)[:, int(np.floor((N - 1) * 0.095))]
        cols = np.concatenate([np.arange(int(N * f), int(N * f) + 8) for f in runs])
        est_r = np.sort(K[:, cols], axis=1)[:, 2]
        rows_err.append(np.log2(np.maximum(true_r, 1e-30) / np.maximum(est_r, 1e-30)))
    for name, err in (("columns", np.concatenate(cols_err)), ("rows", np.concatenate(rows_err))):
        print("%-8s lines %d  log2 error percentiles (0.01, 1, 50, 99, 99.99): %s  outside [-0.75, +1.25]: %.3f  "
              "outside [-0.5, +0.5]: %.3f" % (name, len(err), np.percentile(err, [0.01, 1, 50, 99, 99.99]).round(3),
                                               np.mean((err < -0.75) | (err > 1.25)), np.mean(np.abs(err) > 0.5)))


if __name__ == "__main__":
    main()
