"""CPU tests of the plugin layer's host logic (no GPU): dataset CSV paths, feature files,
the CoverAlgorithm pair driver (enumeration order, symmetrisation, persistence, evaluation)
and its multi-rank path over gloo (world 2 must equal world 1 bitwise)."""
import os
import socket

import numpy as np
import pytest

from acoss import features_io, synthetic, utils
from acoss.algorithms.algorithm_template import CoverAlgorithm


def test_create_dataset_filepaths(tmp_path):
    csv = tmp_path / "d.csv"
    csv.write_text("work_id,track_id\nW1,T1\nW1,T2\nW2,T3\n")
    assert utils.create_dataset_filepaths(str(csv), "root/", ".h5") == ["root/W1/T1.h5", "root/W1/T2.h5",
                                                                         "root/W2/T3.h5"]
    bad = tmp_path / "b.csv"
    bad.write_text("work,track_id\nW1,T1\n")
    with pytest.raises(IOError):
        utils.create_dataset_filepaths(str(bad), "root/")
    assert len(utils.create_dataset_filepaths(utils.COVERS_80_CSV, "x/")) == 164
    assert len(utils.create_dataset_filepaths(utils.DA_TACOS_BENCHMARK_CSV, "x/")) == 15000


def test_feature_file_roundtrip(tmp_path):
    f = {"hpcp": np.arange(24, dtype=np.float32).reshape(2, 12), "label": "W7", "track_id": "T9",
         "madmom_features": {"onsets": np.array([1, 5, 9])}}
    p = str(tmp_path / "W7" / "T9.h5")
    features_io.save_features(p, f)
    g = features_io.load_features(p)
    np.testing.assert_array_equal(g["hpcp"], f["hpcp"])
    assert g["label"] == "W7" and g["track_id"] == "T9"
    np.testing.assert_array_equal(g["madmom_features"]["onsets"], [1, 5, 9])
    with pytest.raises(IOError):
        features_io.load_features(str(tmp_path / "missing.h5"))


class Pairwise(CoverAlgorithm):
    """A deterministic stand-in similarity: score(i, j) = f(i, j), not symmetric."""

    def similarity(self, idxs):
        idxs = np.asarray(idxs)
        s = np.sin(idxs[:, 0] * 1.7 + idxs[:, 1] * 0.3).astype(np.float32)
        for key in self.Ds:
            self.Ds[key][idxs[:, 0], idxs[:, 1]] = s


def _dataset(tmp_path, n_cliques=6):
    rng = np.random.default_rng(0)
    tracks, labels = [], []
    for c in range(n_cliques):
        for _ in range(2 + (c % 2)):
            tracks.append(rng.random((50, 12)).astype(np.float32))
            labels.append(c)
    return synthetic.write_feature_dataset(str(tmp_path), tracks, labels)


@pytest.mark.parametrize("symmetric", [True, False])
def test_all_pairwise_driver(tmp_path, symmetric, monkeypatch):
    monkeypatch.chdir(tmp_path)
    csv, fdir = _dataset(tmp_path)
    a = Pairwise(csv, name="Fake", datapath=fdir, shortname="t", cachedir=str(tmp_path / "cache"),
                 similarity_types=["main", "other"])
    a.all_pairwise(symmetric=symmetric)
    n = a.N
    i, j = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    f = np.sin(i * 1.7 + j * 0.3).astype(np.float32)
    if symmetric:
        f = np.triu(f, 1)
        f = f + f.T
    else:
        np.fill_diagonal(f, 0)
    np.testing.assert_array_equal(np.asarray(a.Ds["main"]), f)
    # cliques were recorded in index order with the CSV's work ids
    assert list(a.cliques) == ["W%05d" % c for c in range(6)]
    stats = a.getEvalStatistics("main")
    assert os.path.exists("results_t_Fake.csv")
    # persisted matrices reload with precomputed=True
    b = Pairwise(csv, name="Fake", datapath=fdir, shortname="t", cachedir=str(tmp_path / "cache"),
                 similarity_types=["main", "other"])
    b.all_pairwise(precomputed=True)
    np.testing.assert_array_equal(np.asarray(b.Ds["main"]), f)
    assert b.getEvalStatistics("main")[3] == stats[3]
    a.cleanup_memmap()
    assert not os.path.exists("%s_main_dmat" % a.get_cacheprefix())


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class PairwiseEvery(Pairwise):
    """The same scorer with Ds assembled on every rank (the late-fusion subclasses' setting)."""
    _Ds_on_every_rank = True


def _rank_worker(rank, world, port, csv, fdir, cache, out, symmetric, every):
    import json
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    cls = PairwiseEvery if every == "class" else Pairwise
    a = cls(csv, name="Fake", datapath=fdir, shortname="w", cachedir=cache, similarity_types=["main", "other"])
    if every == "optin":  # a caller that reads Ds on every rank
        a.Ds_on_every_rank = True
    a.all_pairwise(symmetric=symmetric)
    raised = None
    try:
        np.save(out % rank, np.asarray(a.Ds["main"]))
    except RuntimeError as e:  # gathered onto rank 0 only: reading it elsewhere is an error
        raised = str(e)
    stats = [a.getEvalStatistics(k) for k in ("main", "other")]
    with open((out % rank) + ".json", "w") as f:
        json.dump({"holds": a._holds_Ds, "raised": raised, "keys": sorted(a.Ds),
                   "stats": [[float(v) for v in st[:4]] + [list(map(int, st[4]))] for st in stats]}, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("every", ["", "class", "optin"])
@pytest.mark.parametrize("symmetric", [True, False])
def test_all_pairwise_gloo_world2_equals_world1(tmp_path, symmetric, every, monkeypatch):
    """Two gloo ranks through all_pairwise + getEvalStatistics: rank 0's Ds
    equals the world-1 run bitwise; with the gather (every="", Serra09 / SiMPle) rank 1 holds no
    matrix and reading one raises a RuntimeError that says so instead of returning
    zeros; with the all-gather (the late-fusion algorithms' class setting, or a caller's
    Ds_on_every_rank = True) it holds the same one; both ranks return the same statistics, exactly
    ONE results row per similarity type is written (rank 0), and rank 1 leaves no memmap file
    behind."""
    import json
    import torch.multiprocessing as mp
    monkeypatch.chdir(tmp_path)
    csv, fdir = _dataset(tmp_path, n_cliques=9)
    one = Pairwise(csv, name="One", datapath=fdir, shortname="w", cachedir=str(tmp_path / "c1"))
    one.all_pairwise(symmetric=symmetric)
    ref_stats = [float(v) for v in one.getEvalStatistics("main")[:4]]
    out = str(tmp_path / "rank%d.npy")
    cache = str(tmp_path / "c2")
    mp.start_processes(_rank_worker, args=(2, _free_port(), csv, fdir, cache, out, symmetric, every),
                       nprocs=2, join=True, start_method="spawn")
    np.testing.assert_array_equal(np.load(out % 0), np.asarray(one.Ds["main"]))
    info = [json.load(open((out % r) + ".json")) for r in range(2)]
    if every:
        np.testing.assert_array_equal(np.load(out % 1), np.asarray(one.Ds["main"]))
        assert info[1]["raised"] is None
    else:
        assert not os.path.exists(out % 1)
        assert "gathered onto rank 0 only" in info[1]["raised"] and info[1]["keys"] == ["main", "other"]
    assert info[0]["raised"] is None
    assert info[0]["holds"] and info[1]["holds"] == bool(every)
    assert info[0]["stats"] == info[1]["stats"]
    assert info[0]["stats"][0][:4] == ref_stats
    rows = open("results_w_Fake.csv").read().strip().splitlines()
    assert len(rows) == 3 and rows[0].startswith("name,"), rows  # header + one row per type
    assert sorted(r.split(",")[0] for r in rows[1:]) == ["Fake_main", "Fake_other"], rows
    assert not [f for f in os.listdir(cache) if ".rank" in f]


def test_bind_local_device_rule(monkeypatch):
    """acoss.distributed.bind_local_device under a mocked nccl job: a rank on the
    default device is moved to LOCAL_RANK % device_count; a rank already on its GPU, or bound by
    the caller to another non-default GPU, stays; gloo and uninitialised jobs bind nothing; without
    LOCAL_RANK the launcher fallbacks, then rank % device_count, are used."""
    import torch
    import torch.distributed as dist
    from acoss import distributed as D
    state = {"cur": 0, "set": []}
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: state["cur"])

    def set_device(d):
        state["set"].append(d)
        state["cur"] = d
    monkeypatch.setattr(torch.cuda, "set_device", set_device)
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    backend = {"b": "nccl"}
    monkeypatch.setattr(dist, "get_backend", lambda *a: backend["b"])
    monkeypatch.setattr(dist, "get_rank", lambda *a: 11)
    for v in D.LOCAL_RANK_VARS:
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert D.bind_local_device() == 3 and state["set"] == [3]
    assert D.bind_local_device() == 3 and state["set"] == [3]        # already there: no rebind
    monkeypatch.setenv("LOCAL_RANK", "13")
    state["cur"] = 0
    assert D.bind_local_device() == 5                               # 13 % 8
    state["cur"], state["set"] = 6, []
    assert D.bind_local_device() == 6 and state["set"] == []        # the caller's own binding stays
    monkeypatch.delenv("LOCAL_RANK")
    state["cur"] = 0
    monkeypatch.setenv("SLURM_LOCALID", "2")
    assert D.bind_local_device() == 2
    monkeypatch.delenv("SLURM_LOCALID")
    state["cur"] = 0
    assert D.bind_local_device() == 3                               # rank 11 % 8
    backend["b"] = "gloo"
    state["cur"], state["set"] = 0, []
    assert D.bind_local_device() is None and state["set"] == []
    monkeypatch.setattr(dist, "is_initialized", lambda: False)
    backend["b"] = "nccl"
    assert D.bind_local_device() is None and state["set"] == []


def test_precomputed_world2_binds_before_loading(tmp_path, monkeypatch):
    """all_pairwise(precomputed=True) under a world-2 job binds the rank's GPU BEFORE
    it loads Ds and returns, so the evaluation's first "cuda" allocation lands on the local GPU; a
    rank that holds no matrix skips normalize's device finish."""
    from acoss.algorithms import algorithm_template as T
    monkeypatch.chdir(tmp_path)
    csv, fdir = _dataset(tmp_path)
    a = Pairwise(csv, name="Fake", datapath=fdir, shortname="p", cachedir=str(tmp_path / "cache"))
    a.all_pairwise(symmetric=True)
    calls = []
    monkeypatch.setattr(T, "_dist_info", lambda: (2, 1))
    monkeypatch.setattr(T._dist, "bind_local_device", lambda: calls.append("bind") or 1)
    orig = T.CoverAlgorithm._load_Ds

    def load(self, prefix):
        calls.append("load")
        return orig(self, prefix)
    monkeypatch.setattr(T.CoverAlgorithm, "_load_Ds", load)
    b = Pairwise(csv, name="Fake", datapath=fdir, shortname="p", cachedir=str(tmp_path / "cache"))
    b.all_pairwise(precomputed=True)
    assert calls == ["bind", "load"]
    np.testing.assert_array_equal(np.asarray(b.Ds["main"]), np.asarray(a.Ds["main"]))
    b._holds_Ds = False
    b._finish_device(np.ones(b.N), "serra09")  # returns before touching torch.cuda (no GPU here)


def test_resize_block_shapes():
    from acoss.algorithms.earlyfusion_traile import resize_block
    X = np.random.default_rng(1).random((500, 20))
    for i1, i2, f in [(0, 100, 50), (10, 30, 50), (100, 480, 40)]:
        r = resize_block(X, i1, i2, f)
        assert r.shape == (f, 20) and np.all(np.isfinite(r))
    # a constant block stays constant away from the zero-filled edges
    r = resize_block(np.ones((400, 3)), 100, 300, 50)
    np.testing.assert_allclose(r[10:40], 1.0, rtol=1e-12)


def test_coverid_dispatch_errors(tmp_path, monkeypatch):
    from acoss import coverid
    monkeypatch.chdir(tmp_path)
    with pytest.raises(NotImplementedError):
        coverid.benchmark("x.csv", "y/", algorithm="NoSuchAlgorithm")
    assert coverid.algorithm_names == ["Serra09", "EarlyFusionTraile", "LateFusionChen", "FTM2D", "SiMPle"]
