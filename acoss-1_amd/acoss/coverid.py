"""Benchmark entry point (acoss/coverid.py): `benchmark(...)` and `algorithm_names`.

Same dispatch and call sequence per algorithm as the reference (coverid.py:22-148). Two
reference defects are not reproduced: "EarlyFusionTraile" dispatches
(the reference only matches "EarlyFusion", :72), and `parallel` does not crash (the pairs
are batched on the GPU; with torch.distributed initialised every rank takes a stripe).
FTM2D is outside this engine's scope and raises NotImplementedError.
"""
import argparse
import sys
import time

from .utils import log

__all__ = ['benchmark', 'algorithm_names']

_LOG_FILE_PATH = "acoss.coverid.log"

algorithm_names = ["Serra09", "EarlyFusionTraile", "LateFusionChen", "FTM2D", "SiMPle"]


def benchmark(dataset_csv, feature_dir, feature_type="hpcp", algorithm="Serra09", shortname="covers80",
              parallel=True, n_workers=-1, cachedir="cache"):
    """Run one cover-ID algorithm over a dataset CSV and print/write its evaluation statistics.
    Returns the algorithm object (its Ds hold the similarity matrices)."""
    logger = log(_LOG_FILE_PATH)
    if algorithm not in algorithm_names and algorithm != "EarlyFusion":
        warn = ("acoss.coverid: Couldn't find '%s' algorithm in acoss Available cover id algorithms are %s "
                % (algorithm, str(algorithm_names)))
        logger.debug(warn)
        raise NotImplementedError(warn)
    logger.info("Running acoss cover identification benchmarking for the algorithm - '%s'" % algorithm)
    start = time.monotonic()
    kw = dict(dataset_csv=dataset_csv, datapath=feature_dir, chroma_type=feature_type, shortname=shortname,
              cachedir=cachedir)
    if algorithm == "Serra09":
        from .algorithms.rqa_serra09 import Serra09
        algo = Serra09(**kw)
        logger.info('Computing pairwise similarity...')
        algo.all_pairwise(parallel, n_cores=n_workers, symmetric=True)
        algo.normalize_by_length()
    elif algorithm in ("EarlyFusionTraile", "EarlyFusion"):
        from .algorithms.earlyfusion_traile import EarlyFusion
        algo = EarlyFusion(**kw)
        # the reference's load_features(i) loop (coverid.py:80-81): the same per-song caches and clique
        # bookkeeping, with the uncached songs' block features made ceil(N / 256) launches at a time
        algo.prepare()
        logger.info('Feature loading done...')
        logger.info('Computing pairwise similarity...')
        algo.all_pairwise(parallel, n_cores=n_workers, symmetric=True)
        algo.do_late_fusion()
    elif algorithm == "LateFusionChen":
        from .algorithms.latefusion_chen import ChenFusion
        algo = ChenFusion(**kw)
        logger.info('Computing pairwise similarity...')
        algo.all_pairwise(parallel, n_cores=n_workers, symmetric=True)
        algo.normalize_by_length()
        algo.do_late_fusion()
    elif algorithm == "SiMPle":
        from .algorithms.simple_silva import Simple
        algo = Simple(**kw)
        algo.prepare()
        logger.info('Feature loading done...')
        logger.info('Computing pairwise similarity...')
        algo.all_pairwise(parallel, n_cores=n_workers, symmetric=False)
    else:
        raise NotImplementedError("FTM2D is outside the scope of the MI355X engine (DESIGN.md)")
    logger.info('Running benchmark evaluations on the given dataset - %s' % dataset_csv)
    for similarity_type in list(algo.Ds.keys()):
        algo.getEvalStatistics(similarity_type)
    algo.cleanup_memmap()
    logger.info("acoss.coverid benchmarking finished in %s" % (time.monotonic() - start))
    logger.info("Log file located at '%s'" % _LOG_FILE_PATH)
    return algo


def parser_args(cmd_args):
    parser = argparse.ArgumentParser(sys.argv[0], description="Benchmark a specific cover id algorithm with a given "
                                                              "input dataset csv annotations",
                                     formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    parser.add_argument("-i", '--dataset_csv', type=str, action="store", help="Input dataset csv file")
    parser.add_argument("-d", '--feature_dir', type=str, action="store", default='../features_covers80',
                        help="Path to data files")
    parser.add_argument("-m", "--method", type=str, action="store", default="Serra09", help="Algorithm name")
    parser.add_argument("-s", "--shortname", type=str, action="store", default="covers80", help="Dataset short name")
    parser.add_argument("-c", '--chroma_type', type=str, action="store", default="hpcp",
                        help="Type of chroma to use for experiments")
    parser.add_argument("-p", '--parallel', type=int, choices=(0, 1), action="store", default=1,
                        help="Accepted for compatibility")
    parser.add_argument("-n", '--n_workers', type=int, action="store", default=-1, help="Accepted for compatibility")
    return parser.parse_args(cmd_args)


if __name__ == '__main__':
    args = parser_args(sys.argv[1:])
    benchmark(dataset_csv=args.dataset_csv, feature_dir=args.feature_dir, feature_type=args.chroma_type,
              algorithm=args.method, shortname=args.shortname, parallel=bool(args.parallel), n_workers=args.n_workers)
