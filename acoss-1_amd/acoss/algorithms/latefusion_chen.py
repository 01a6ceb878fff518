"""ChenFusion — late fusion of Qmax and Dmax (acoss/algorithms/latefusion_chen.py), MI355X engine.

Chen, N., Li, W. and Xiao, H., 2018. Fusing similarity functions for cover song
identification. Multimedia Tools and Applications, 77(2), pp.2629-2652.

One acoss_crp_align call per chunk produces both alignments of the same CRP (serra09 ->
Ds['qmax'], chen17 -> Ds['dmax']), :58-73; SNF late fusion runs on the device
(utils/similarity_fusion.py).
"""
import argparse

import numpy as np

from .algorithm_template import CoverAlgorithm
from .rqa_serra09 import ChromaBackedAlgorithm
from .utils.similarity_fusion import doSimilarityFusion

__all__ = ["ChenFusion"]


class ChenFusion(ChromaBackedAlgorithm):
    # the SNF late fusion runs on every rank (row-sharded): every rank needs the assembled Ds
    _Ds_on_every_rank = True

    def __init__(self, dataset_csv, datapath, chroma_type='hpcp', shortname='benchmark', oti=True, kappa=0.095,
                 tau=1, m=9, downsample_fac=40, cachedir="cache"):
        self._init_chroma(chroma_type, oti, kappa, tau, m, downsample_fac)
        CoverAlgorithm.__init__(self, dataset_csv, name="LateFusionChen", similarity_types=["qmax", "dmax"],
                                datapath=datapath, shortname=shortname, cachedir=cachedir)

    def similarity(self, idxs):
        idxs = np.asarray(idxs)
        if len(idxs) == 0:
            return
        r = self._score(idxs, dmax=True)
        self.Ds["qmax"][idxs[:, 0], idxs[:, 1]] = r["qmax"]
        self.Ds["dmax"][idxs[:, 0], idxs[:, 1]] = r["dmax"]

    def _device_scores(self, idxs):
        return self._score_dev(idxs, dmax=True)

    def normalize_by_length(self):
        """D[i, j] = sqrt(n_j) / D[i, j] (latefusion_chen.py:75-85): float64 quotient stored in
        float32; a zero score gives inf, as in the reference (acoss_ds_finish mode 'chen')."""
        self._finish_device(self._norm_factors(), "chen")

    def do_late_fusion(self):
        """SNF of all Ds (K=20, 20 iterations), then back to larger-is-closer (:87-91)."""
        DLate = doSimilarityFusion([self.Ds[s] for s in self.Ds], K=20, niters=20, reg_diag=1)[1]
        for key in self.Ds:
            self.Ds[key] *= -1
        self.Ds["Late"] = DLate


if __name__ == '__main__':
    parser = argparse.ArgumentParser(description="Benchmarking with Chen's late fusion cover id algorithm",
                                     formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    parser.add_argument("-i", '--dataset_csv', type=str, action="store", help="Input dataset csv file")
    parser.add_argument("-d", '--datapath', type=str, action="store", default='../features_covers80',
                        help="Path to data files")
    parser.add_argument("-s", "--shortname", type=str, action="store", default="Covers80",
                        help="Short name for dataset")
    parser.add_argument("-c", '--chroma_type', type=str, action="store", default='hpcp',
                        help="Type of chroma to use for experiments")
    parser.add_argument("-p", '--parallel', type=int, choices=(0, 1), action="store", default=0,
                        help="Ignored: pairs are batched on the GPU")
    parser.add_argument("-n", '--n_cores', type=int, action="store", default=1, help="Ignored")
    cmd_args = parser.parse_args()
    chenFusion = ChenFusion(dataset_csv=cmd_args.dataset_csv, datapath=cmd_args.datapath,
                            chroma_type=cmd_args.chroma_type, shortname=cmd_args.shortname)
    chenFusion.all_pairwise(cmd_args.parallel, cmd_args.n_cores, symmetric=True)
    chenFusion.normalize_by_length()
    chenFusion.do_late_fusion()
    for similarity_type in chenFusion.Ds.keys():
        print(similarity_type)
        chenFusion.getEvalStatistics(similarity_type)
    chenFusion.cleanup_memmap()
    print("... Done ....")
