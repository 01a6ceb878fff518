"""Device-resident song banks and the batched pair scorers built on the C-ABI.

A bank packs every track of a corpus once into HBM (one contiguous (sum n, 12) float32
block + offsets/lengths, SURVEY.md §8f row 3 layout); the scorers then take (P, 2) pair
index lists and return one score per pair, computed by the HIP kernels in a single
stream-ordered call. This replaces the reference's per-pair Python loop
(CoverAlgorithm.similarity, acoss/algorithms/algorithm_template.py:121-140 and the plugin
overrides) with one batched call per pair chunk.
"""
import numpy as np

from . import _lib
from .synthetic import pack


def stacked_len(n, m=9, tau=1):
    """essentia stackChromaFrames count (crp.hip stacked_len)."""
    inc = m * tau
    return 0 if n <= inc else (n - inc + tau - 1) // tau


class ChromaBank:
    """12-bin chroma of a whole corpus resident on the current GPU."""

    def __init__(self, tracks=None, packed=None):
        """tracks: list of (n_i, 12) arrays, or packed=(feats (sum n, 12) f32 device tensor,
        frame offsets, lengths) already resident in HBM."""
        torch = _lib._torch()
        if packed is not None:
            feats, off, lens = packed
            self.lens = np.asarray(lens, np.int32)
            self.feats = feats
            self.off = torch.as_tensor(np.asarray(off, np.int64)).cuda()
        else:
            feats, off, lens = pack([np.asarray(t, np.float32) for t in tracks])
            self.lens = lens
            self.feats = torch.as_tensor(feats).cuda()
            self.off = torch.as_tensor(off).cuda()
        self.n_tracks = len(self.lens)
        self.max_len = int(self.lens.max()) if len(self.lens) else 0
        self.len = torch.as_tensor(self.lens).cuda()

    def crp_align(self, pairs, m=9, tau=1, kappa=0.095, oti=True, gamma_open=0.5, gamma_ext=0.5, qmax=True,
                  dmax=False, want_oti=False):
        """Serra09 (Qmax) / Chen (dmax) scores for (query, reference) pairs."""
        torch = _lib._torch()
        # host pairs stay on the host until _lib.crp_align checks them there and uploads them
        # without a stream synchronisation (chunk after chunk keeps the GPU busy)
        pairs = np.asarray(pairs, np.int32).reshape(-1, 2) if not isinstance(pairs, torch.Tensor) else pairs
        if (pairs.size if isinstance(pairs, np.ndarray) else pairs.numel()) == 0:
            z = torch.zeros(0, dtype=torch.float32, device="cuda")
            return {k: z for k, on in (("qmax", qmax), ("dmax", dmax), ("oti", want_oti)) if on}
        short = []
        if stacked_len(int(self.lens.min()), m, tau) <= 0:  # only then can a pair hold a short track
            hp = pairs if isinstance(pairs, np.ndarray) else pairs.cpu().numpy()
            short = [i for i in np.unique(hp) if stacked_len(self.lens[i], m, tau) <= 0]
        if short:
            raise ValueError("tracks %s are too short for frameStackSize=%d, frameStackStride=%d (essentia raises)"
                             % (short[:5], m, tau))
        params = _lib.crp_params(m, tau, kappa, oti, gamma_open, gamma_ext)
        return _lib.crp_align(self.feats, self.off, self.len, self.max_len, pairs, params, qmax=qmax,
                              dmax=dmax, oti=want_oti)
