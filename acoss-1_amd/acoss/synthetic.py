"""Synthetic HPCP-like cover-song corpora (SURVEY.md §8d "Synthetic inputs").

There is no network and no audio in this environment, so benchmarks and end-to-end tests
run on seeded synthetic 12-d chroma with the clique structure of the real datasets:

* per clique a base sequence: a random walk over the 24 major/minor triad templates
  (dwell ~U[8, 64] frames) plus |N(0, 0.1)| noise, non-negative, unit-max per frame
  (like essentia HPCP), with 2 % silent (all-zero) frames;
* every cover = the base rolled by a random key k in [0, 12), time-stretched by
  U[0.8, 1.25] (nearest-index resampling), fresh noise, renormalised; float32 (n, 12).

Clique shapes: covers80 (164 tracks: 77x2, 2x3, 1x4, from acoss/data/covers80_annotations.csv)
and Da-TACOS benchmark (1000x13 + 2000 singletons = 15,000 tracks).
"""
import os

import numpy as np

SEED = 20250101
_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def triad_templates():
    """(24, 12) major + minor triads, unit max."""
    T = np.zeros((24, 12), np.float32)
    for r in range(12):
        T[r, [r, (r + 4) % 12, (r + 7) % 12]] = 1.0
        T[12 + r, [r, (r + 3) % 12, (r + 7) % 12]] = 1.0
    return T


def _unitmax(x):
    mx = x.max(axis=1, keepdims=True)
    return np.where(mx > 0, x / np.where(mx > 0, mx, 1), 0).astype(np.float32)


def base_sequence(rng, n, silence=0.02):
    T = triad_templates()
    out = np.empty((n, 12), np.float32)
    i = 0
    while i < n:
        dwell = int(rng.integers(8, 65))
        out[i:i + dwell] = T[rng.integers(0, 24)]
        i += dwell
    return out


def render(rng, base, silence=0.02):
    x = base + np.abs(rng.normal(0.0, 0.1, base.shape)).astype(np.float32)
    x = _unitmax(x)
    x[rng.random(len(x)) < silence] = 0.0
    return x


def cover_of(rng, base, n_out=None, stretch=(0.8, 1.25)):
    k = int(rng.integers(0, 12))
    s = float(rng.uniform(*stretch))
    n = n_out if n_out is not None else max(16, int(round(len(base) * s)))
    idx = np.minimum((np.arange(n) * (len(base) / n)).astype(np.int64), len(base) - 1)
    return np.roll(base[idx], k, axis=1)


def clique_sizes(shape):
    if shape == "covers80":
        import pandas as pd
        df = pd.read_csv(os.path.join(_DATA, "covers80_annotations.csv"), dtype=str)
        return [int(c) for c in df.groupby("work_id", sort=False).size().values]
    if shape == "datacos":
        return [13] * 1000 + [1] * 2000
    raise ValueError(shape)


def make_corpus(shape="covers80", frames=2000, frames_jitter=0.0, seed=SEED, stretch=True):
    """Return (tracks: list of (n_i, 12) float32, labels: int array).

    frames: length of every base sequence (the CSM input length); with
    stretch=True covers are resampled to U[0.8,1.25]x that length, else all tracks have
    exactly `frames` frames. frames_jitter: base length ~ U[1-j, 1+j] * frames.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    tracks, labels = [], []
    for lab, size in enumerate(clique_sizes(shape)):
        n0 = frames if frames_jitter <= 0 else int(round(frames * rng.uniform(1 - frames_jitter, 1 + frames_jitter)))
        base = base_sequence(rng, n0)
        for v in range(size):
            if v == 0:
                seq = base
            else:
                seq = cover_of(rng, base, None if stretch else n0)
            tracks.append(render(rng, seq))
            labels.append(lab)
    return tracks, np.asarray(labels, np.int32)


# A corpus on which the score ranks are not saturated (MAP well below 1), so a MAP/MR1
# comparison between two score matrices can detect a difference (SURVEY §8d "MAP parity").
# Unrelated songs share chord phrases from one global pool (a progression of 4-8 triads with
# its own dwells), and covers are partial, locally re-harmonised, noisier excerpts.
HARD = {"pool": 24, "phrases": (3, 8), "noise": 0.3, "stretch": (0.7, 1.4), "excerpt": (0.5, 1.0),
        "substitute": 0.25}


def _phrase_pool(rng, n_phrases):
    pool = []
    for _ in range(n_phrases):
        k = int(rng.integers(4, 9))
        pool.append((rng.integers(0, 24, size=k), rng.integers(8, 41, size=k)))
    return pool


def _hard_base(rng, n, pool, per_song):
    """A song = a few phrases of the shared pool (its own pick and order, transposed by one
    random key per phrase), repeated until n frames."""
    T = triad_templates()
    picks = rng.choice(len(pool), size=per_song, replace=False)
    keys = rng.integers(0, 12, size=per_song)
    out = np.empty((n, 12), np.float32)
    i, p = 0, 0
    while i < n:
        chords, dwells = pool[picks[p % per_song]]
        key = int(keys[p % per_song])
        for c, d in zip(chords, dwells):
            if i >= n:
                break
            c = int(c)
            root, minor = (c % 12 + key) % 12, c // 12
            out[i:i + int(d)] = T[root + 12 * minor]
            i += int(d)
        p += 1
    return out


def _hard_cover(rng, base, n_out, params):
    T = triad_templates()
    lo, hi = params["excerpt"]
    frac = float(rng.uniform(lo, hi))
    seg = max(16, int(round(len(base) * frac)))
    st = int(rng.integers(0, len(base) - seg + 1))
    part = base[st:st + seg].copy()
    # re-harmonise: each chord run is replaced by a random triad with probability `substitute`
    edges = np.flatnonzero(np.any(part[1:] != part[:-1], axis=1)) + 1
    bounds = np.concatenate([[0], edges, [len(part)]])
    for a, b in zip(bounds[:-1], bounds[1:]):
        if rng.random() < params["substitute"]:
            part[a:b] = T[int(rng.integers(0, 24))]
    if n_out is None:
        n_out = max(16, int(round(len(base) * float(rng.uniform(*params["stretch"])))))
    idx = np.minimum((np.arange(n_out) * (len(part) / n_out)).astype(np.int64), len(part) - 1)
    return np.roll(part[idx], int(rng.integers(0, 12)), axis=1)


def make_hard_corpus(shape="covers80", frames=2000, seed=SEED, fixed_length=True, params=None):
    """(tracks, labels) of the discriminative corpus (HARD). fixed_length: every track has
    exactly `frames` frames (the bench's metric config, M = N = frames); else covers are
    stretched by params['stretch']."""
    params = dict(HARD, **(params or {}))
    rng = np.random.Generator(np.random.PCG64(seed))
    pool = _phrase_pool(rng, params["pool"])
    tracks, labels = [], []
    for lab, size in enumerate(clique_sizes(shape)):
        base = _hard_base(rng, frames, pool, int(rng.integers(params["phrases"][0], params["phrases"][1] + 1)))
        for v in range(size):
            seq = base if v == 0 else _hard_cover(rng, base, frames if fixed_length else None, params)
            x = seq + np.abs(rng.normal(0.0, params["noise"], seq.shape)).astype(np.float32)
            x = _unitmax(x)
            x[rng.random(len(x)) < 0.02] = 0.0
            tracks.append(x)
            labels.append(lab)
    return tracks, np.asarray(labels, np.int32)


def pack(tracks):
    """List of (n_i, 12) -> (feats (sum n, 12) f32, off int64, len int32)."""
    lens = np.array([len(t) for t in tracks], np.int32)
    off = np.zeros(len(tracks), np.int64)
    if len(tracks) > 1:
        off[1:] = np.cumsum(lens[:-1])
    feats = np.ascontiguousarray(np.concatenate(tracks, 0), np.float32) if tracks else np.zeros((0, 12), np.float32)
    return feats, off, lens


def write_feature_dataset(root, tracks, labels, with_mfcc=False, seed=SEED, beat_period=43, mfcc_shortfall=43,
                          chroma_keys=("hpcp", "crema", "chroma_cens"), mfcc_from_chroma=False):
    """Write a dataset the plugin classes can read: '<root>/dataset.csv' (work_id, track_id)
    and one feature file per track at '<root>/features/<work_id>/<track_id>.npz' with the keys
    of the reference's feature dicts (README.md:93-114): the chroma_keys ('hpcp', 'crema',
    'chroma_cens', each the same array), 'label', 'track_id', and with_mfcc: 'mfcc_htk' (20, n - mfcc_shortfall) and
    'madmom_features/onsets' (a fixed beat grid with jitter, up to the chroma's last frame). The
    reference extractor's mfcc_htk has about 43 frames fewer than its hpcp (22050-sample windows
    with validFrameThresholdRatio=1, acoss/features.py:884), so the last beats fall past the
    MFCC's end as in real feature files. mfcc_from_chroma: the MFCC frames are one fixed random
    projection of the chroma frames plus noise (covers then share MFCC structure, so the MFCC
    scores separate cliques too); otherwise independent noise. Returns (csv path, feature dir with
    trailing slash)."""
    from .features_io import save_features
    rng = np.random.Generator(np.random.PCG64(seed))
    proj = rng.standard_normal((20, 12)).astype(np.float32) if mfcc_from_chroma else None
    feat_dir = os.path.join(root, "features") + "/"
    rows = []
    for k, (t, lab) in enumerate(zip(tracks, labels)):
        work, track = "W%05d" % int(lab), "T%06d" % k
        t = np.asarray(t, np.float32)
        f = dict({k: t for k in chroma_keys}, label=work, track_id=track)
        if with_mfcc:
            n = len(t)
            nm = max(1, n - mfcc_shortfall)
            if proj is not None:
                f["mfcc_htk"] = (proj @ t[:nm].T + 0.3 * rng.standard_normal((20, nm))).astype(np.float32)
            else:
                f["mfcc_htk"] = rng.standard_normal((20, nm)).astype(np.float32)
            beats = np.arange(0, n - 1, beat_period) + rng.integers(0, 3, size=len(range(0, n - 1, beat_period)))
            f["madmom_features"] = {"onsets": np.unique(np.clip(beats, 0, n - 1)).astype(np.int64)}
        save_features(feat_dir + work + "/" + track + ".h5", f)
        rows.append((work, track))
    csv = os.path.join(root, "dataset.csv")
    with open(csv, "w") as fo:
        fo.write("work_id,track_id\n")
        for w, tr in rows:
            fo.write("%s,%s\n" % (w, tr))
    return csv, feat_dir
