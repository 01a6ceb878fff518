"""SiMPle — similarity matrix profile (acoss/algorithms/simple_silva.py), MI355X engine.

Silva, Yeh, Batista, Keogh. SiMPle: Assessing music similarity using subsequences joins.
ISMIR 2016.

`prepare()` computes every track's SiMPle features once on the GPU (features.hip: window
means, Hann smoothing, column L2 norm; the reference recomputes them for every pair,
:120-126), and `similarity(idxs)` scores a chunk of ordered pairs with one acoss_simple_mp
call (simple.hip: Simple.oti + matrix profile + median). Ds['main'][i, j] = -median(MP).
"""
import argparse

import numpy as np

from .. import _lib
from .algorithm_template import CoverAlgorithm

__all__ = ["Simple"]


class Simple(CoverAlgorithm):
    def __init__(self, dataset_csv, datapath, chroma_type='hpcp', shortname='Covers80', SSLEN=10, WIN=200,
                 SKIP=100, cachedir="cache"):
        self.SSLEN = SSLEN
        self.WIN = WIN
        self.SKIP = SKIP
        self.chroma_type = chroma_type
        self.all_feats = {}
        self._packed = None
        CoverAlgorithm.__init__(self, dataset_csv=dataset_csv, name="SiMPle", datapath=datapath, shortname=shortname,
                                cachedir=cachedir)

    def _features(self, chromas):
        from ..synthetic import pack
        feats, off, lens = pack([np.asarray(c, np.float32) for c in chromas])
        return _lib.simple_features(feats, off, lens, win=self.WIN, skip=self.SKIP)

    def load_features(self, i, do_plot=False):
        """(12, floor(n / SKIP)) float64 SiMPle features of song i (simple_silva.py:34-43)."""
        if i not in self.all_feats:
            feats = CoverAlgorithm.load_features(self, i)
            out, _, T = self._features([feats[self.chroma_type]])
            self.all_feats[i] = out.cpu().numpy().reshape(12, int(T[0]))
        return self.all_feats[i]

    def prepare(self):
        if self._prepared:
            return
        chromas = [f[self.chroma_type] for f in self.load_features_many((self.chroma_type,))]
        out, out_off, T = self._features(chromas)
        host = out.cpu().numpy()
        for i in range(self.N):
            self.all_feats[i] = host[out_off[i]:out_off[i] + 12 * T[i]].reshape(12, int(T[i]))
        self._packed = (out, out_off, T)
        self._prepared = True

    def track_lengths(self):
        self.prepare()
        return np.maximum(self._packed[2].astype(np.int64), 1)

    def oti(self, seq_a, seq_b):
        """(roll(seq_b, k*), argsort of the 12 shift scores) (simple_silva.py:45-54)."""
        pa, pb = np.sum(seq_a, 1), np.sum(seq_b, 1)
        v = np.array([np.dot(pa, np.roll(pb, i, axis=0)) for i in range(12)])
        order = np.argsort(v, kind="stable")
        return np.roll(seq_b, order[-1], axis=0), order

    def simple_sim(self, seq_a, seq_b):
        """median of the matrix profile of seq_a against seq_b (simple_silva.py:68-118), on the GPU."""
        score, _ = _lib.simple_mp([seq_a, seq_b], np.array([[0, 1]], np.int32), self.SSLEN, apply_oti=False)
        return float(score.cpu().numpy()[0])

    def similarity(self, idxs):
        idxs = np.asarray(idxs)
        if len(idxs) == 0:
            return
        self.prepare()
        out, off, T = self._packed
        score, _ = _lib.simple_mp_packed(out, off, T, idxs.astype(np.int32), self.SSLEN)
        self.Ds['main'][idxs[:, 0], idxs[:, 1]] = -score.cpu().numpy()

    def _device_scores(self, idxs):
        """-median(MP) per ordered pair as float32 device scores (the memmap's dtype)."""
        idxs = np.asarray(idxs)
        self.prepare()
        out, off, T = self._packed
        score, _ = _lib.simple_mp_packed(out, off, T, idxs.astype(np.int32), self.SSLEN)
        return {'main': (-score).float()}


if __name__ == '__main__':
    parser = argparse.ArgumentParser(description="Benchmarking with Similarity Matrix Profile-based similarity",
                                     formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    parser.add_argument("-i", '--dataset_csv', type=str, action="store", help="Input dataset csv file")
    parser.add_argument("-d", '--datapath', type=str, action="store", default='features_covers80',
                        help="Path to data files")
    parser.add_argument("-s", "--shortname", type=str, action="store", default="Covers80", help="Short name for dataset")
    parser.add_argument("-c", '--chroma_type', type=str, action="store", default='crema',
                        help="Type of chroma to use for experiments")
    parser.add_argument("-p", '--parallel', type=int, choices=(0, 1), action="store", default=0, help="Ignored")
    parser.add_argument("-n", '--n_cores', type=int, action="store", default=1, help="Ignored")
    cmd_args = parser.parse_args()
    simple = Simple(dataset_csv=cmd_args.dataset_csv, datapath=cmd_args.datapath, chroma_type=cmd_args.chroma_type,
                    shortname=cmd_args.shortname)
    simple.all_pairwise(cmd_args.parallel, cmd_args.n_cores, symmetric=False)
    for similarity_type in simple.Ds.keys():
        simple.getEvalStatistics(similarity_type)
    simple.cleanup_memmap()
    print("... Done ....")
