"""One rank of tests/test_gpu_multirank.py (not a test module): runs a plugin's real HIP
all_pairwise under torch.distributed (gloo; the ranks share one GPU) and rank 0 saves Ds.
Usage: python tests/multirank_worker.py ALGO CSV FEATURE_DIR CACHEDIR OUT.npz
(RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT from the environment). ALGO "bench:<name>" runs
coverid.benchmark(algorithm=<name>) instead of the plugin calls. ACOSS_MR_DOWNSAMPLE: Serra09's
downsample_fac (default: the reference's); ACOSS_MR_SIMPLE_WIN / _SKIP: SiMPle's WIN / SKIP on
crema (default: the reference's hpcp, 200 / 100); ACOSS_MR_DIGEST=1: save a SHA-256 of every Ds matrix
(and its shape) instead of the matrix (the 15,000-song runs)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "acoss-1_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    algo, csv, fdir, cachedir, out = sys.argv[1:6]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(0)
    if world > 1:
        dist.init_process_group("gloo")
    os.makedirs(cachedir, exist_ok=True)
    os.chdir(cachedir)
    if algo.startswith("bench:"):
        # the whole reference entry point (coverid.py:22-148): all_pairwise, normalisation, late
        # fusion, getEvalStatistics on every key (only rank 0 writes results_mr_<name>.csv, in the
        # cachedir: this process's cwd), cleanup_memmap
        from acoss import coverid
        a = coverid.benchmark(csv, fdir, algorithm=algo.split(":", 1)[1], shortname="mr", cachedir=cachedir)
    elif algo == "Serra09":
        from acoss.algorithms.rqa_serra09 import Serra09
        kw = {}
        if os.environ.get("ACOSS_MR_DOWNSAMPLE"):
            kw["downsample_fac"] = int(os.environ["ACOSS_MR_DOWNSAMPLE"])
        a = Serra09(csv, fdir, shortname="mr", cachedir=cachedir, **kw)
        a.all_pairwise(symmetric=True)
        a.normalize_by_length()
    elif algo in ("ChenFusion", "ChenLate"):
        from acoss.algorithms.latefusion_chen import ChenFusion
        a = ChenFusion(csv, fdir, shortname="mr", cachedir=cachedir)
        a.all_pairwise(symmetric=True)
        if algo == "ChenLate":
            # SNF late fusion (latefusion_chen.py:87-91): row-sharded across the ranks
            a.normalize_by_length()
            a.do_late_fusion()
    elif algo == "EarlyFusion":
        # config 5's flow (coverid.py:72-88): block features, the four scores of the stripe on the
        # device, one all-gather per score, then SNF late and early+late (row-sharded when
        # ACOSS_SNF_SHARD=1)
        from acoss.algorithms.earlyfusion_traile import EarlyFusion
        a = EarlyFusion(csv, fdir, shortname="mr", cachedir=cachedir)
        a.prepare()
        a.all_pairwise(symmetric=True)
        a.do_late_fusion()
    else:
        from acoss.algorithms.simple_silva import Simple
        kw = {}
        if os.environ.get("ACOSS_MR_SIMPLE_WIN"):  # (window / hop of the SiMPle features)
            kw = {"chroma_type": "crema", "WIN": int(os.environ["ACOSS_MR_SIMPLE_WIN"]),
                  "SKIP": int(os.environ["ACOSS_MR_SIMPLE_SKIP"])}
        a = Simple(csv, fdir, shortname="mr", cachedir=cachedir, **kw)
        a.all_pairwise(symmetric=False)
    if rank == 0:
        if os.environ.get("ACOSS_MR_DIGEST") == "1":
            import hashlib
            dig = {}
            for k, v in a.Ds.items():
                arr = np.ascontiguousarray(np.asarray(v))
                dig[k] = np.array([hashlib.sha256(arr.tobytes()).hexdigest(), str(arr.shape),
                                   str(int(np.isfinite(arr).sum()))])
            np.savez(out, **dig)
        else:
            np.savez(out, **{k: np.asarray(v) for k, v in a.Ds.items()})
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
