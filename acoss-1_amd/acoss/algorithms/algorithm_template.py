"""CoverAlgorithm — the plugin base class (acoss/algorithms/algorithm_template.py), MI355X engine.

The public surface is the reference's: constructor arguments, `filepaths`, `cliques`, `N`,
`Ds` (float32 N x N memmaps at '<cachedir>/<name>_<shortname>_<type>_dmat'),
`load_features(i)`, `get_all_clique_ids()`, `similarity(idxs)`, `all_pairwise(parallel,
n_cores, symmetric, precomputed)`, `cleanup_memmap()`, `getEvalStatistics(type, topsidx)`.

What changes is how the pair loop runs (algorithm_template.py:142-193). The reference calls
`similarity` on one pair (serial) or on 45 chunks (joblib processes). Here:
  * `prepare()` loads every track once (clique bookkeeping in index order, as the serial
    reference does) and lets the subclass build its device-resident banks;
  * the pairs, in the reference's enumeration order (combinations / permutations), go to
    `similarity` in large chunks; the subclasses score a chunk with one batched HIP call;
  * with torch.distributed initialised (one process per GPU, RCCL), every rank is bound to its
    local rank's GPU (acoss.distributed.bind_local_device), scores one cost-balanced row stripe
    and ONE exchange assembles Ds: a gather onto rank 0 for the scorers that rank 0 alone
    finishes (Serra09, SiMPle), an all-gather onto every rank for those whose SNF late fusion
    runs on every rank next (`_Ds_on_every_rank`: ChenFusion, EarlyFusion); `parallel` /
    `n_cores` are accepted for signature compatibility and ignored;
  * subclasses with a HIP scorer (`_device_scores`) keep the stripe on the device: the
    all-gather, `Ds += Ds.T` and the subclasses' normalize_by_length run as HIP kernels
    (finish.hip), and getEvalStatistics ranks on the device (acoss_eval_ranks), so no O(N^2)
    host loop is left for Da-TACOS-sized runs;
  * every rank keeps Ds in a file-backed memmap of its own (rank 0: the reference's file, other
    ranks '<file>.rank<r>', unlinked as soon as it is mapped, so it never outlives the process),
    and only rank 0 prints the statistics and writes the results CSV and the Ds file, so ranks
    never write one file (the reference's single shared memmap and results file, :172-177,
    :277-290); ranks that do not hold Ds get rank 0's statistics from getEvalStatistics;
  * Ds is saved as '<prefix>_Ds.h5' (the reference's file, :163,193; one dataset per
    similarity type, as deepdish lays out a dict) when h5py is importable, and always as the
    '<prefix>_Ds.npz' twin; `precomputed=True` reads either back.
Reference defects not reproduced: the NameError of parallel=True at
:174-192 and `cleanup_memmap` calling rmtree on files (:202).
"""
import os
import warnings

import numpy as np

from .. import distributed as _dist
from .. import evaluation
from ..features_io import load_features as _load_feature_file
from ..utils import create_dataset_filepaths

__all__ = ["CoverAlgorithm"]

PAIR_CHUNK = 1 << 20  # pairs per similarity() call (the engine batches further inside)


def _dist_info():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(), dist.get_rank()
    except ImportError:
        pass
    return 1, 0


def _on_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except ImportError:
        return False


class _RootOnlyDs(dict):
    """Ds on a rank > 0 after a gather onto rank 0 (Serra09, SiMPle under torch.distributed): the
    similarity types are still listed, but reading a matrix raises instead of silently returning
    the zeros of a matrix this rank never received. The memmaps are dropped, which
    frees their unlinked files' disk blocks."""

    def __init__(self, Ds, rank):
        dict.__init__(self, {k: None for k in Ds})
        self._rank = rank

    def __getitem__(self, key):
        if key not in self:
            raise KeyError(key)
        raise RuntimeError(
            "Ds[%r] was gathered onto rank 0 only; rank %d does not hold it. Read Ds on rank 0, or set "
            "algorithm.Ds_on_every_rank = True before all_pairwise to all-gather it onto every rank "
            "(INTEGRATION.md section 3)." % (key, self._rank))

    def values(self):
        return [self[k] for k in self]  # raises on the first key

    def items(self):
        return [(k, self[k]) for k in self]


class CoverAlgorithm(object):
    def __init__(self, dataset_csv, name="Serra09", datapath="features_benchmark", shortname="full",
                 cachedir="cache", similarity_types=["main"]):
        self.name = name
        self.shortname = shortname
        self.cachedir = cachedir
        self.filepaths = create_dataset_filepaths(dataset_csv, root_audio_dir=datapath, file_format=".h5")
        self.cliques = {}
        self.N = len(self.filepaths)
        os.makedirs(cachedir, exist_ok=True)
        self.Ds = {}
        _, rank = _dist_info()
        for s in similarity_types:
            self.Ds[s] = self._new_dmat(s, rank)
        self._prepared = False
        self._holds_Ds = True         # this rank's Ds hold the assembled matrices
        self._stats_from_root = False  # getEvalStatistics takes rank 0's statistics (world > 1)
        if rank == 0:
            print("Initialized %s algorithm on %i songs in dataset %s" % (name, self.N, shortname))

    # Ds assembled on every rank (all-gather) instead of rank 0 only (gather): subclasses whose
    # late fusion runs on every rank after all_pairwise (ChenFusion, EarlyFusion) set this
    _Ds_on_every_rank = False
    # the same, opted into by a caller that reads Ds on every rank (an instance attribute)
    Ds_on_every_rank = False

    def _new_dmat(self, s, rank):
        """Ds[s] as a float32 (N, N) memmap (:61). Rank r > 0's file is unlinked once mapped: the
        mapping stays valid (POSIX), the disk blocks are freed when the process ends, and nothing
        is left in cachedir (0.9 GB per matrix and rank at Da-TACOS size)."""
        path = self._dmat_path(s, rank)
        mm = np.memmap(path, shape=(self.N, self.N), mode="w+", dtype="float32")
        if rank != 0:
            try:
                os.remove(path)
            except OSError:
                pass
        return mm

    # ------------------------------------------------------------------ features
    def get_cacheprefix(self):
        return "%s/%s_%s" % (self.cachedir, self.name, self.shortname)

    def _dmat_path(self, s, rank=0):
        """The memmap file of Ds[s] (:61). Ranks other than 0 keep their copy of the assembled
        matrix in a file of their own ('.rank<r>'), so no two ranks write one file and no rank
        holds N x N float32 per similarity type in RAM (0.9 GB each at Da-TACOS size)."""
        base = "%s_%s_dmat" % (self.get_cacheprefix(), s)
        return base if rank == 0 else "%s.rank%d" % (base, rank)

    def load_features(self, i):
        """Feature dict of song i; records its clique as a side effect (:70-94)."""
        feats = _load_feature_file(self.filepaths[i])
        self._record_clique(i, feats["label"])
        return feats

    def _record_clique(self, i, label):
        if label not in self.cliques:
            self.cliques[label] = set([])
        self.cliques[label].add(i)

    def load_features_many(self, keys):
        """The `keys` entries (plus 'label') of every song's feature file, read on a thread pool,
        in song order; records the cliques as load_features does."""
        from ..features_io import load_many
        out = load_many(self.filepaths, keys=tuple(keys) + ("label",))
        for i, f in enumerate(out):
            self._record_clique(i, f["label"])
        return out

    def get_all_clique_ids(self, verbose=False):
        """Clique membership of every song, cached in '<prefix>_clique_info.txt' (:96-119)."""
        path = "%s_clique_info.txt" % self.get_cacheprefix()
        if not os.path.exists(path):
            with open(path, "w") as fout:
                for i in range(len(self.filepaths)):
                    feats = CoverAlgorithm.load_features(self, i)
                    if verbose:
                        print(i)
                    fout.write("%i,%s\n" % (i, feats["label"]))
        else:
            with open(path) as fin:
                for line in fin.readlines():
                    i, label = line.split(",")
                    label = label.strip()
                    self.cliques.setdefault(label, set([])).add(int(i))

    def prepare(self):
        """Load every song once (index order) and build the subclass's device banks."""
        if not self._prepared:
            for i in range(self.N):
                self.load_features(i)
            self._prepared = True

    def track_lengths(self):
        """Per-song cost proxy for the stripe balance (frames at the pair kernel's input)."""
        return np.ones(self.N, np.int64) * 100

    # ------------------------------------------------------------------ pairs
    def similarity(self, idxs):
        """Score the (P, 2) pairs into Ds (base class: zeros, :121-140)."""
        idxs = np.asarray(idxs)
        for key in self.Ds:
            self.Ds[key][idxs[:, 0], idxs[:, 1]] = 0.0

    def _device_scores(self, idxs):
        """Subclasses with a HIP scorer return {similarity type: float32 CUDA tensor (P,)} for the
        (P, 2) pairs; the base class has none (None: the host `similarity` loop is used)."""
        return None

    def all_pairwise(self, parallel=0, n_cores=12, symmetric=False, precomputed=False):
        prefix = self.get_cacheprefix()
        world, rank = _dist_info()
        if world > 1:  # before ANY "cuda" allocation, the precomputed path's evaluation included
            _dist.bind_local_device()
        if precomputed:
            self._load_Ds(prefix)
            self.get_all_clique_ids()
            self._holds_Ds, self._stats_from_root = True, False
            return
        self.prepare()
        if world > 1:
            bounds = _dist.stripe_bounds(self.track_lengths(), world, symmetric, m=0, tau=0)
        else:
            bounds = [(0, self.N)]
        r0, r1 = bounds[rank]
        every = world == 1 or self._Ds_on_every_rank or self.Ds_on_every_rank
        self._holds_Ds = every or rank == 0
        self._stats_from_root = not every
        if not self._device_all_pairwise(bounds, r0, r1, world, symmetric, every):
            for chunk in self._pair_chunks(r0, r1, symmetric):
                self.similarity(chunk)
            if world > 1:
                self._gather_stripes(bounds, r0, r1, every)
            if symmetric and self._holds_Ds:
                for key in self.Ds:
                    self.Ds[key] += self.Ds[key].T
        if not self._holds_Ds:  # reading Ds here is a caller error: make it a loud one
            self.Ds = _RootOnlyDs(self.Ds, rank)
        if rank == 0:
            self._save_Ds(prefix)

    def _pair_chunks(self, r0, r1, symmetric):
        """The stripe's pairs in the reference's enumeration order (combinations / permutations,
        :168-171), PAIR_CHUNK at a time, with a progress line on stderr about every 10 s (the
        reference prints progress in its serial loop, :179-187)."""
        import sys
        import time
        n_pairs = sum(self.N - i - 1 if symmetric else self.N - 1 for i in range(r0, r1))
        t0 = last = time.perf_counter()
        done = 0
        for chunk in _dist.stripe_pair_chunks(self.N, r0, r1, symmetric, PAIR_CHUNK):
            yield chunk
            done += len(chunk)
            now = time.perf_counter()
            if now - last >= 10.0 and done < n_pairs:
                last = now
                print("%s: %d / %d pairs, %.1f s" % (self.name, done, n_pairs, now - t0), file=sys.stderr, flush=True)

    def _device_all_pairwise(self, bounds, r0, r1, world, symmetric, every=True):
        """The pair loop with the stripe kept in HBM: score chunks on the device, scatter into
        the (r1 - r0, N) stripe, one exchange (world > 1: all-gather if `every`, else a gather onto
        rank 0), symmetrise with acoss_ds_finish and copy into Ds on the ranks that receive the
        matrix. Returns False if the subclass has no device scorer."""
        if type(self)._device_scores is CoverAlgorithm._device_scores:
            return False
        import torch
        from .. import _lib
        blocks = {k: torch.zeros((r1 - r0, self.N), dtype=torch.float32, device="cuda") for k in self.Ds}
        for chunk in self._pair_chunks(r0, r1, symmetric):
            sc = self._device_scores(chunk)
            p = torch.from_numpy(np.ascontiguousarray(chunk, np.int32)).pin_memory().to("cuda", non_blocking=True).long()
            for k in blocks:
                blocks[k][p[:, 0] - r0, p[:, 1]] = sc[k]
        for k in list(blocks):
            blk = blocks.pop(k)
            if world == 1:
                full = blk
            elif every:
                full = _dist.all_gather_stripes(blk, bounds)
            else:
                full = _dist.gather_stripes(blk, bounds, dst=0)
            del blk
            if full is None:  # not the root of the gather
                continue
            if symmetric:
                _lib.ds_finish(full, symmetric=True)
            self.Ds[k][:] = full.cpu().numpy()
            del full  # one assembled matrix on the device at a time
        return True

    def _gather_stripes(self, bounds, r0, r1, every=True):
        import torch
        dev = "cuda" if torch.cuda.is_available() else "cpu"
        for key in self.Ds:
            blk = torch.as_tensor(np.array(self.Ds[key][r0:r1])).to(dev)
            full = _dist.all_gather_stripes(blk, bounds) if every else _dist.gather_stripes(blk, bounds, dst=0)
            if full is not None:
                self.Ds[key][:] = full.cpu().numpy()

    def _finish_device(self, norm, mode):
        """normalize_by_length on the device for every Ds key (acoss_ds_finish, mode 'serra09' or
        'chen'): one upload, one HIP kernel, one download per matrix. A rank that does not hold
        the gathered matrices has nothing to normalise."""
        if not self._holds_Ds:
            return
        from .. import _lib
        torch = _lib._torch()  # binds this rank's GPU (nccl) before the first "cuda" allocation
        norm = np.asarray(norm, np.float64)
        for key in list(self.Ds):
            D = torch.as_tensor(np.ascontiguousarray(self.Ds[key], np.float32)).cuda()
            _lib.ds_finish(D, norm, symmetric=False, mode=mode)
            self.Ds[key][:] = D.cpu().numpy()

    def _save_Ds(self, prefix):
        """'<prefix>_Ds.h5' (h5py, one float32 dataset per similarity type) when h5py is
        importable, and always the '<prefix>_Ds.npz' twin."""
        mats = {k: np.asarray(v) for k, v in self.Ds.items()}
        np.savez("%s_Ds.npz" % prefix, **mats)
        try:
            import h5py
        except ImportError:
            return
        from ..features_io import save_h5
        save_h5("%s_Ds.h5" % prefix, mats, h5py)

    def _load_Ds(self, prefix):
        """The reference reads '<prefix>_Ds.h5' (:164-166); here the .h5 when h5py is importable,
        else the .npz twin."""
        npz, h5 = "%s_Ds.npz" % prefix, "%s_Ds.h5" % prefix
        if os.path.exists(h5):
            try:
                from ..features_io import _load_h5
                self.Ds = {k: np.asarray(v, np.float32) for k, v in _load_h5(h5).items()}
                return
            except ImportError:
                pass
        with np.load(npz, allow_pickle=False) as z:
            self.Ds = {k: np.array(z[k]) for k in z.files}

    def cleanup_memmap(self):
        """Delete the memmap files of Ds (:195-203)."""
        _, rank = _dist_info()
        for s in list(self.Ds):
            path = self._dmat_path(s, rank)
            try:
                if os.path.exists(path):
                    os.remove(path)
            except OSError:
                print("Could not clean-up automatically.")

    # ------------------------------------------------------------------ evaluation
    def getEvalStatistics(self, similarity_type, topsidx=[1, 10, 100, 1000]):
        """MR, MRR, MDR, MAP, Top-k of Ds[similarity_type] (:206-291); prints them and appends
        a row to 'results_<shortname>_<name>.csv'. Under torch.distributed only rank 0 prints and
        writes the row (one row per call, as the reference's single process writes). When Ds was
        gathered onto rank 0 only, rank 0 computes the statistics and broadcasts them, so every rank
        must call this (coverid.benchmark does) and every rank returns the same values: a
        collective call, like the gather before it. Set
        `Ds_on_every_rank = True` before all_pairwise to all-gather Ds onto every rank instead;
        each rank then evaluates on its own, without any collective here."""
        world, rank = _dist_info()
        stats = None
        if self._holds_Ds and (rank == 0 or not self._stats_from_root):
            stats = self._eval_stats(similarity_type, topsidx)
        if world > 1 and self._stats_from_root:
            import torch.distributed as dist
            box = [stats]
            dist.broadcast_object_list(box, src=0)
            stats = box[0]
        MR, MRR, MDR, MAP, tops = stats
        if rank == 0:
            if np.isnan(MR):
                warnings.warn("no clique with at least two songs")
            print("%s %s STATS\n-------------------------\nMR = %.3g\nMRR = %.3g\nMDR = %.3g\nMAP = %.3g"
                  % (self.name, similarity_type, MR, MRR, MDR, MAP))
            for t, v in zip(topsidx, tops):
                print("Top-%i: %i" % (t, v))
            evaluation.write_results_csv("results_%s_%s.csv" % (self.shortname, self.name), self.name,
                                         similarity_type, stats, topsidx)
        return MR, MRR, MDR, MAP, tops

    def _eval_stats(self, similarity_type, topsidx):
        D = np.array(self.Ds[similarity_type], dtype=np.float32)
        cliques = [sorted(self.cliques[s]) for s in self.cliques]
        if _on_gpu():  # the O(N^2) rank step as a HIP kernel (same statistics, same host code)
            from .. import _lib
            torch = _lib._torch()  # binds this rank's GPU (nccl) before the first "cuda" allocation
            return evaluation.eval_statistics_device(torch.as_tensor(D).cuda(), cliques=cliques, topsidx=topsidx)
        return evaluation.eval_statistics_cliques(D, cliques, topsidx)  # the reference's host computation
