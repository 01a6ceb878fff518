"""Serra09 — cross recurrence quantification (acoss/algorithms/rqa_serra09.py), MI355X engine.

Serra, J., Serra, X., & Andrzejak, R. G. (2009). Cross recurrence quantification for cover
song identification. New Journal of Physics, 11(9), 093017.

Per pair the reference builds essentia ChromaCrossSimilarity(frameStackSize=m,
frameStackStride=tau, binarizePercentile=kappa, oti) and CoverSongSimilarity('serra09',
'symmetric') and stores Qmax (:55-69). Here `prepare()` median-downsamples every track on
the GPU (features.hip) into one packed HBM block, and `similarity(idxs)` scores a whole chunk
of pairs with one acoss_crp_align call (crp_split.hip / crp.hip).
"""
import argparse
import sys

import numpy as np

from .. import _lib
from ..engine import ChromaBank
from .algorithm_template import CoverAlgorithm

__all__ = ["Serra09", "ChromaBackedAlgorithm"]


class ChromaBackedAlgorithm(CoverAlgorithm):
    """Shared by Serra09 and ChenFusion: cached median-downsampled chroma + a device bank."""

    def _init_chroma(self, chroma_type, oti, kappa, tau, m, downsample_fac):
        self.oti = oti
        self.tau = tau
        self.m = m
        self.chroma_type = chroma_type
        self.kappa = kappa
        self.downsample_fac = downsample_fac
        self.all_feats = {}  # i -> downsampled chroma (n_i, 12) float32, as the reference caches
        self._bank = None

    def _downsample(self, chromas):
        from ..synthetic import pack
        feats, off, lens = pack([np.asarray(c, np.float32) for c in chromas])
        out, out_off, out_len = _lib.median_downsample(feats, off, lens, self.downsample_fac)
        return out, out_off, out_len

    def load_features(self, i):
        """Median-downsampled chroma of song i (rqa_serra09.py:44-53), cached."""
        if i not in self.all_feats:
            feats = CoverAlgorithm.load_features(self, i)
            out, _, _ = self._downsample([feats[self.chroma_type]])
            self.all_feats[i] = out.cpu().numpy()
        return self.all_feats[i]

    def prepare(self):
        if self._prepared:
            return
        chromas = [f[self.chroma_type] for f in self.load_features_many((self.chroma_type,))]
        out, out_off, out_len = self._downsample(chromas)
        host = out.cpu().numpy()
        for i in range(self.N):
            self.all_feats[i] = host[out_off[i]:out_off[i] + out_len[i]]
        self._bank = ChromaBank(packed=(out, out_off, out_len))
        self._prepared = True

    def track_lengths(self):
        self.prepare()
        return np.maximum(self._bank.lens.astype(np.int64) - self.m * self.tau, 1)

    def _score_dev(self, idxs, dmax=False):
        self.prepare()
        return self._bank.crp_align(np.asarray(idxs, np.int32), m=self.m, tau=self.tau, kappa=self.kappa,
                                    oti=self.oti, qmax=True, dmax=dmax)

    def _score(self, idxs, dmax=False):
        return {k: v.cpu().numpy() for k, v in self._score_dev(idxs, dmax).items()}

    def _norm_factors(self):
        """sqrt(n_j) in float64, n_j = downsampled frames of song j."""
        return np.sqrt(np.array([self.load_features(j).shape[0] for j in range(self.N)], np.float64))


class Serra09(ChromaBackedAlgorithm):
    def __init__(self, dataset_csv, datapath, chroma_type='hpcp', shortname='benchmark', oti=True, kappa=0.095,
                 tau=1, m=9, downsample_fac=40, cachedir="cache"):
        self._init_chroma(chroma_type, oti, kappa, tau, m, downsample_fac)
        CoverAlgorithm.__init__(self, dataset_csv=dataset_csv, name="Serra09", datapath=datapath, shortname=shortname,
                                cachedir=cachedir)

    def similarity(self, idxs):
        """Qmax of every (query, reference) pair into every Ds key (rqa_serra09.py:55-69)."""
        idxs = np.asarray(idxs)
        if len(idxs) == 0:
            return
        q = self._score(idxs)["qmax"]
        for key in self.Ds.keys():
            self.Ds[key][idxs[:, 0], idxs[:, 1]] = q

    def _device_scores(self, idxs):
        q = self._score_dev(idxs)["qmax"]
        return {key: q for key in self.Ds}

    def normalize_by_length(self):
        """D[i, j] /= sqrt(n_j), n_j = downsampled frames of song j (rqa_serra09.py:71-83);
        the quotient is taken in float64 and stored in the float32 matrix, as the reference
        (acoss_ds_finish mode 'serra09')."""
        self._finish_device(self._norm_factors(), "serra09")


def parser_args(args):
    parser = argparse.ArgumentParser(sys.argv[0], description="Benchmarking with Joan Serra's Cover id algorithm",
                                     formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    parser.add_argument("-i", '--dataset_csv', type=str, action="store", help="Input dataset csv file")
    parser.add_argument("-d", '--datapath', type=str, action="store", help="Path to data files")
    parser.add_argument("-s", "--shortname", type=str, action="store", default="covers80",
                        help="Short name for dataset")
    parser.add_argument("-c", '--chroma_type', type=str, action="store", default="hpcp",
                        help="Type of chroma to use for experiments")
    parser.add_argument("-p", '--parallel', type=int, choices=(0, 1), action="store", default=0,
                        help="Parallel computing or not (ignored: pairs are batched on the GPU)")
    parser.add_argument("-n", '--n_cores', type=int, action="store", default=1, help="Ignored (see --parallel)")
    return parser.parse_args(args)


if __name__ == '__main__':
    cmd_args = parser_args(sys.argv[1:])
    # keyword arguments: the reference passes these positionally in the wrong order (:108)
    serra09 = Serra09(dataset_csv=cmd_args.dataset_csv, datapath=cmd_args.datapath,
                      chroma_type=cmd_args.chroma_type, shortname=cmd_args.shortname)
    serra09.all_pairwise(cmd_args.parallel, cmd_args.n_cores, symmetric=True)
    serra09.normalize_by_length()
    for similarity_type in serra09.Ds.keys():
        print(similarity_type)
        serra09.getEvalStatistics(similarity_type)
    serra09.cleanup_memmap()
    print("... Done ....")
