"""CPU tests of the host side: the C-ABI library's exports (no compute call), evaluation
statistics vs the reference's golden outputs, corpus shapes, row-stripe sharding and the
world_size-2 all-gather of stripes over gloo."""
import os
import re
import socket

import numpy as np
import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def gold():
    from conftest import GOLDEN
    return np.load(GOLDEN)


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "acoss_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(acoss_\w+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from acoss import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libacoss_hip.so not built (run __graft_entry__.build())")
    lib = _lib.load_library()
    names = _header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    # every header function with an int return is bound with argtypes in the wrapper
    for n in names:
        if n not in ("acoss_version", "acoss_last_error", "acoss_profile_phase_name"):
            assert n in _lib.SIGNATURES, n
    assert lib.acoss_version().decode().startswith("acoss-mi355x")


def test_product_path_has_no_cpu_fallback():
    import torch
    from acoss import _lib
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.AcossHipError):
        _lib.crp_align(np.zeros((20, 12), np.float32), [0], [20], 20, np.zeros((0, 2), np.int32), _lib.crp_params())


@pytest.mark.parametrize("tag", ["eval_c80", "eval_dt"])
def test_eval_statistics_golden(gold, tag, tmp_path):
    from acoss import evaluation
    MR, MRR, MDR, MAP, tops = evaluation.eval_statistics(gold[tag + "_D"], gold[tag + "_labels"])
    np.testing.assert_allclose([MR, MRR, MDR, MAP], gold[tag + "_stats"], rtol=1e-12, atol=1e-15)
    np.testing.assert_array_equal(tops, gold[tag + "_tops"])
    f = tmp_path / "res.csv"
    evaluation.write_results_csv(str(f), "Golden", "main", (MR, MRR, MDR, MAP, tops))
    assert f.read_text().splitlines()[-1] == str(gold[tag + "_csv"]).splitlines()[-1]


def test_corpus_shapes():
    from acoss import synthetic
    sizes = synthetic.clique_sizes("covers80")
    assert sum(sizes) == 164
    assert sorted(np.bincount(sizes)[2:].tolist()) == sorted([77, 2, 1])
    tracks, labels = synthetic.make_corpus("covers80", frames=100, seed=1)
    assert len(tracks) == 164 and len(labels) == 164
    assert all(t.dtype == np.float32 and t.shape[1] == 12 for t in tracks)
    assert all(np.all(t >= 0) and np.all(t.max(1) <= 1.0) for t in tracks)


@pytest.mark.parametrize("symmetric", [True, False])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_stripes_cover_all_pairs(world, symmetric):
    from acoss import distributed
    rng = np.random.default_rng(world)
    lens = rng.integers(20, 400, size=57)
    bounds = distributed.stripe_bounds(lens, world, symmetric)
    assert bounds[0][0] == 0 and bounds[-1][1] == 57
    assert all(b[1] == c[0] for b, c in zip(bounds, bounds[1:]))
    allp = np.concatenate([distributed.stripe_pairs(57, r0, r1, symmetric) for r0, r1 in bounds])
    n_expect = 57 * 56 // 2 if symmetric else 57 * 56
    assert len(allp) == n_expect == len({tuple(p) for p in allp.tolist()})
    if world > 1:
        costs = [distributed.row_costs(lens, symmetric)[r0:r1].sum() for r0, r1 in bounds]
        assert max(costs) <= 1.35 * (sum(costs) / world) + distributed.row_costs(lens, symmetric).max()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, n, out_path):
    import torch
    import torch.distributed as dist
    from acoss import distributed
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    lens = np.full(n, 100)
    bounds = distributed.stripe_bounds(lens, world, True)
    r0, r1 = bounds[rank]
    pairs = distributed.stripe_pairs(n, r0, r1, True)
    scores = torch.as_tensor((pairs[:, 0] * 1000 + pairs[:, 1]).astype(np.float32))
    blk = distributed.scatter_stripe(pairs, scores, r0, r1, n)
    full = distributed.all_gather_stripes(blk, bounds)
    if rank == 0:
        np.save(out_path, full.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_all_gather_world2(tmp_path):
    import torch.multiprocessing as mp
    n = 23
    out = str(tmp_path / "full.npy")
    mp.start_processes(_gloo_worker, args=(2, _free_port(), n, out), nprocs=2, join=True, start_method="spawn")
    full = np.load(out)
    i, j = np.triu_indices(n, 1)
    expect = np.zeros((n, n), np.float32)
    expect[i, j] = i * 1000 + j
    np.testing.assert_array_equal(full, expect)
