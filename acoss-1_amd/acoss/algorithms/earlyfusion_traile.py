"""EarlyFusion — early MFCC/HPCP fusion (acoss/algorithms/earlyfusion_traile.py), MI355X engine.

Tralie, C.J., 2017. Early mfcc and hpcp fusion for robust cover song identification.
arXiv preprint arXiv:1707.04680.

Per pair (A15, :157-198) everything runs on the GPU through the C-ABI: three CSMs on MFMA
(euclidean on the MFCC blocks and on the SSM blocks, blocked-OTI cosine on the chroma
blocks), kappa-NN binarisation, getWCSM of each CSM, their sum -> exp(-sum) -> binarisation,
and the four constrained Smith-Waterman alignments of a chunk in one launch.

The beat-synchronous block features (load_features, :67-154) are computed
on the GPU too (efblocks.hip acoss_ef_block_features: every block of a batch of tracks in one
launch, skimage's resize restated in float64), batched over all songs in prepare() and cached on
disk as the reference does. `resize_block` (:214-247) stays as the reference's public helper: it
restates skimage >= 0.19 `resize(..., anti_aliasing=True, mode='constant')` (Gaussian pre-filter
with sigma = max(0, (factor - 1) / 2), then a grid-mode linear zoom with zero fill) with
scipy.ndimage. skimage is absent here, so both restatements are pinned against each other and
against an independent loop restatement (tests/test_earlyfusion_host.py), not against skimage.
"""
import argparse
import os
import time

import numpy as np

from .. import _lib
from ..features_io import load_features as _load_feature_file
from ..features_io import save_features as _save_feature_file
from .algorithm_template import CoverAlgorithm
from .utils.cross_recurrence import nneighbs
from .utils.similarity_fusion import doSimilarityFusion

__all__ = ["EarlyFusion", "resize_block"]


def resize_block(X, i1, i2, frames_per_block, median_aggregate=False):
    """Resample X[i1:i2] to frames_per_block rows (earlyfusion_traile.py:214-247)."""
    from scipy import ndimage
    if median_aggregate:
        raise NotImplementedError("median_aggregate=True needs librosa.util.sync (absent); the reference default "
                                  "is False")
    x = np.asarray(X[i1:i2, :], dtype=np.float64)
    factor = x.shape[0] / float(frames_per_block)
    sigma = max(0.0, (factor - 1.0) / 2.0)
    if sigma > 0:
        x = ndimage.gaussian_filter(x, (sigma, 0.0), mode="constant", cval=0.0)
    ret = ndimage.zoom(x, (frames_per_block / float(x.shape[0]), 1.0), order=1, mode="grid-constant", cval=0.0,
                       grid_mode=True)
    ret[np.isinf(ret)] = 0
    ret[np.isnan(ret)] = 0
    return ret


class EarlyFusion(CoverAlgorithm):
    # the SNF late fusion runs on every rank (row-sharded): every rank needs the assembled Ds
    _Ds_on_every_rank = True

    def __init__(self, dataset_csv, datapath, chroma_type='hpcp', shortname='Covers80', blocksize=20,
                 mfccs_per_block=50, ssm_res=50, chromas_per_block=40, kappa=0.1, K=10, niters=5, log_times=False,
                 cachedir="cache"):
        self.chroma_type = chroma_type
        self.blocksize = blocksize
        self.mfccs_per_block = mfccs_per_block
        self.chromas_per_block = chromas_per_block
        self.kappa = kappa
        self.K = K
        self.niters = niters
        self.all_block_feats = {}
        self.log_times = log_times
        if log_times:
            self.times = {'features': [], 'raw': []}
        self._dev = {}
        self._pending = []  # background cache writes (flush_cache)
        CoverAlgorithm.__init__(self, dataset_csv=dataset_csv, name="EarlyFusionTraile", datapath=datapath,
                                shortname=shortname, similarity_types=["mfccs", "ssms", "chromas", "early"],
                                cachedir=cachedir)

    def get_cacheprefix(self):
        return "%s/%s_%s_%s" % (self.cachedir, self.name, self.shortname, self.chroma_type)

    def load_features(self, i, do_plot=False):
        """Blocked features of song i: 'mfccs', 'ssms', 'chromas', 'chroma_med' (:67-154),
        cached in memory and on disk ('<prefix>_<i>.npz'); computed on the GPU."""
        filepath = "%s_%i.h5" % (self.get_cacheprefix(), i)
        if i in self.all_block_feats:
            return self.all_block_feats[i]
        try:
            self.all_block_feats[i] = _load_feature_file(filepath)
            CoverAlgorithm.load_features(self, i)
            return self.all_block_feats[i]
        except IOError:
            pass
        return self._compute_blocks([i])[0]

    def _compute_blocks(self, idx):
        """Block features of songs idx in one acoss_ef_block_features launch; cached in memory and
        on disk like load_features. Under torch.distributed every rank computes the blocks on its
        own GPU (one launch per 256 songs) and only rank 0 writes the disk cache, so W ranks do not
        write the same 15,000 files W times."""
        tic = time.time()
        from ..features_io import load_many
        feats = load_many([self.filepaths[i] for i in idx],
                          keys=(self.chroma_type, "mfcc_htk", "madmom_features", "label"))
        for i, f in zip(idx, feats):
            self._record_clique(i, f["label"])
        chroma = [np.asarray(f[self.chroma_type], np.float32) for f in feats]
        mfcc = [np.array(f['mfcc_htk'], dtype=np.float32).T for f in feats]
        onsets = [np.asarray(f['madmom_features']['onsets'], np.int64) for f in feats]
        out = _lib.ef_block_features(chroma, mfcc, onsets, self.blocksize, self.mfccs_per_block,
                                     self.chromas_per_block)
        host = {k: out[k].cpu().numpy() for k in ("mfccs", "ssms", "chromas", "chroma_med")}
        from .algorithm_template import _dist_info
        write_cache = _dist_info()[1] == 0
        res = []
        for t, i in enumerate(idx):
            b0, nb = int(out["block_off"][t]), int(out["n_blocks"][t])
            bf = {"mfccs": host["mfccs"][b0:b0 + nb], "ssms": host["ssms"][b0:b0 + nb],
                  "chromas": host["chromas"][b0:b0 + nb], "chroma_med": host["chroma_med"][t]}
            self.all_block_feats[i] = bf
            if write_cache:  # on a background thread: ~1 ms of np.savez per song (15 s at 15,000 songs)
                self._pending.append(self._cache_writer().submit(
                    _save_feature_file, "%s_%i.h5" % (self.get_cacheprefix(), i), bf))
            res.append(bf)
        if self.log_times:
            self.times['features'].append((time.time() - tic) / max(1, len(idx)))
        return res

    def _cache_writer(self):
        """One background thread for the block-feature disk cache, so the ~1 ms np.savez per song
        overlaps the GPU work that follows prepare() instead of adding to it. The exit hook holds
        only a weak reference, so it never keeps an instance (its ~2 GB of block features at
        Da-TACOS size, its device tensors) alive."""
        if getattr(self, "_writer", None) is None:
            import atexit
            import weakref
            from concurrent.futures import ThreadPoolExecutor
            self._writer = ThreadPoolExecutor(max_workers=1)
            ref = weakref.ref(self)

            def _flush_at_exit():
                obj = ref()
                if obj is not None:
                    obj.flush_cache()

            self._atexit = _flush_at_exit
            atexit.register(_flush_at_exit)
        return self._writer

    def flush_cache(self):
        """Wait until every block-feature cache file of prepare() is on disk (re-raises the first
        failed write), then stop the writer thread; all_pairwise and interpreter exit call it."""
        pending, self._pending = self._pending, []
        writer, self._writer = getattr(self, "_writer", None), None
        hook = getattr(self, "_atexit", None)
        if hook is not None:
            import atexit
            atexit.unregister(hook)
            self._atexit = None
        try:
            for f in pending:
                f.result()
        finally:
            if writer is not None:
                writer.shutdown(wait=True)

    def all_pairwise(self, *args, **kwargs):
        try:
            out = CoverAlgorithm.all_pairwise(self, *args, **kwargs)
        except BaseException:
            try:  # the scoring error is the one to see; a cache-write error is only chained
                self.flush_cache()
            except Exception as e:  # noqa: BLE001
                import warnings
                warnings.warn("EarlyFusion block-feature cache write failed: %r" % (e,))
            raise
        self.flush_cache()
        return out

    def _device(self, i):
        if i not in self._dev:
            torch = _lib._torch()
            f = self.load_features(i)
            self._dev[i] = {k: torch.as_tensor(np.ascontiguousarray(f[k], np.float32)).cuda()
                            for k in ("mfccs", "ssms", "chromas")}
            self._dev[i]["chroma_med"] = np.asarray(f["chroma_med"], np.float32)
        return self._dev[i]

    def pair_matrices(self, i, j):
        """The four binary matrices of pair (i, j) (device uint8), in score order
        mfccs, ssms, chromas, early (:157-189)."""
        torch = _lib._torch()
        a, b = self._device(i), self._device(j)
        csms = {}
        csms['mfccs'] = _lib.csm(a['mfccs'], b['mfccs'], kind="euclidean")
        csms['ssms'] = _lib.csm(a['ssms'], b['ssms'], kind="euclidean")
        oti = int(_lib.get_oti(a['chroma_med'], b['chroma_med']).item())
        csms['chromas'] = _lib.csm(a['chromas'], b['chromas'], kind="cosine", oti_shift=oti)
        ncols = csms['mfccs'].shape[1]
        nn = nneighbs(self.kappa, ncols)
        mats = [_lib.binarize_rows(csms[s], nn) for s in ('mfccs', 'ssms', 'chromas')]
        wsum = torch.zeros_like(csms['mfccs'])
        for s in ('mfccs', 'ssms', 'chromas'):
            wsum += _lib.wcsm(csms[s], self.K, self.K, 0.5)
        mats.append(_lib.binarize_rows(_lib.neg_exp(wsum), nn))
        return mats

    def _bank(self):
        """All tracks' block features packed once into HBM for the batched kernels."""
        if getattr(self, "_dev_bank", None) is None:
            torch = _lib._torch()
            self.prepare()
            feats = [self.load_features(i) for i in range(self.N)]
            nb = np.array([f["mfccs"].shape[0] for f in feats], np.int32)
            off = np.zeros(self.N, np.int64)
            off[1:] = np.cumsum(nb[:-1])

            def cat(key):
                return torch.as_tensor(np.ascontiguousarray(np.concatenate([f[key] for f in feats]), np.float32)).cuda()

            self._dev_bank = {"mfccs": cat("mfccs"), "ssms": cat("ssms"), "chromas": cat("chromas"),
                              "chroma_med": torch.as_tensor(np.stack([np.asarray(f["chroma_med"], np.float32)
                                                                      for f in feats])).cuda(),
                              "off": torch.as_tensor(off).cuda(), "nb": torch.as_tensor(nb).cuda(), "nb_host": nb,
                              "max_blocks": int(nb.max())}
        return self._dev_bank

    def similarity(self, idxs, do_plot=False):
        """The four scores of every pair, one batched C-ABI call (acoss_earlyfusion)."""
        idxs = np.asarray(idxs)
        if len(idxs) == 0:
            return
        tic = time.time()
        scores = _lib.earlyfusion(self._bank(), idxs.astype(np.int32), self.kappa, self.K).cpu().numpy()
        if self.log_times:
            self.times['raw'].append((time.time() - tic) / len(idxs))
        for s, key in enumerate(("mfccs", "ssms", "chromas", "early")):
            self.Ds[key][idxs[:, 0], idxs[:, 1]] = scores[:, s]

    def _device_scores(self, idxs):
        """The four scores of every pair as float32 device tensors (the memmap's dtype), from one
        acoss_earlyfusion call: all_pairwise keeps the stripe on the device and all-gathers it
        across ranks (algorithm_template._device_all_pairwise)."""
        idxs = np.asarray(idxs)
        tic = time.time()
        sc = _lib.earlyfusion(self._bank(), idxs.astype(np.int32), self.kappa, self.K)
        if self.log_times:
            self.times['raw'].append((time.time() - tic) / max(1, len(idxs)))
        return {key: sc[:, s].float() for s, key in enumerate(("mfccs", "ssms", "chromas", "early"))}

    def track_lengths(self):
        """Beat blocks per song: a pair costs nb_i * nb_j (three CSMs, four SW), so the row
        stripes balance that (acoss.distributed.stripe_bounds with m = tau = 0)."""
        self.prepare()
        return np.array([max(1, self.all_block_feats[i]["mfccs"].shape[0]) for i in range(self.N)], np.int64)

    def prepare(self, chunk=256):
        """Every song's block features: from the memory / disk cache, the rest on the GPU in
        batches of `chunk` songs. The cached block features and the cached songs' labels are read
        by the native reader in two batched calls (features_io.load_many), not one np.load per
        file."""
        if not self._prepared:
            from ..features_io import cache_readable, load_many
            todo = [i for i in range(self.N) if i not in self.all_block_feats]
            paths = {i: "%s_%i.h5" % (self.get_cacheprefix(), i) for i in todo}
            have = [i for i in todo if cache_readable(paths[i])]
            if have:
                for i, bf in zip(have, load_many([paths[i] for i in have])):
                    self.all_block_feats[i] = bf
                for i, f in zip(have, load_many([self.filepaths[i] for i in have], keys=("label",))):
                    self._record_clique(i, f["label"])
            done = set(have)
            missing = [i for i in todo if i not in done]
            for c0 in range(0, len(missing), chunk):
                self._compute_blocks(missing[c0:c0 + chunk])
            self._prepared = True

    def do_late_fusion(self):
        """SNF of 1/(1 + D) for the late and early+late outputs (:200-206)."""
        self.Ds["late"] = doSimilarityFusion([1.0 / (1.0 + self.Ds[s]) for s in ["chromas", "ssms", "mfccs"]], K=20,
                                             niters=20, reg_diag=1)[1]
        self.Ds["early+late"] = doSimilarityFusion([1.0 / (1.0 + self.Ds[s])
                                                    for s in ["chromas", "ssms", "mfccs", "early"]], K=20, niters=20,
                                                   reg_diag=1)[1]


if __name__ == '__main__':
    parser = argparse.ArgumentParser(description="Benchmarking with Early Similarity Network Fusion of HPCP, MFCC, "
                                                 "and MFCC SSMs",
                                     formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    parser.add_argument("-i", '--dataset_csv', type=str, action="store", help="Input dataset csv file")
    parser.add_argument("-d", '--datapath', type=str, action="store", default='../features_covers80',
                        help="Path to data files")
    parser.add_argument("-s", "--shortname", type=str, action="store", default="Covers80", help="Short name for dataset")
    parser.add_argument("-c", '--chroma_type', type=str, action="store", default='hpcp',
                        help="Type of chroma to use for experiments")
    parser.add_argument("-p", '--parallel', type=int, choices=(0, 1), action="store", default=0, help="Ignored")
    parser.add_argument("-n", '--n_cores', type=int, action="store", default=1, help="Ignored")
    parser.add_argument("-l", '--log_times', type=int, choices=(0, 1), action="store", default=0,
                        help="Whether to log times to a file")
    cmd_args = parser.parse_args()
    ef = EarlyFusion(dataset_csv=cmd_args.dataset_csv, datapath=cmd_args.datapath, chroma_type=cmd_args.chroma_type,
                     shortname=cmd_args.shortname, log_times=bool(cmd_args.log_times))
    for i in range(len(ef.filepaths)):
        ef.load_features(i)
    ef.all_pairwise(cmd_args.parallel, cmd_args.n_cores, symmetric=True)
    ef.do_late_fusion()
    for similarity_type in ef.Ds:
        ef.getEvalStatistics(similarity_type)
    ef.cleanup_memmap()
    if ef.log_times:
        for s in ef.times:
            print("%s: %.3g" % (s, np.mean(ef.times[s])))
    print("... Done ....")
