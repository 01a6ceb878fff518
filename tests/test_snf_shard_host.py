"""CPU test of the row-sharded SNF loop's host logic (similarity_fusion._fusion_sharded, SURVEY
§8f row 2) over gloo, world 2 and 3 against world 1. The two HIP halves of a step
(acoss_snf_diffuse_rows / acoss_snf_left_rows) are replaced by an elementwise torch float64
restatement whose every output element is computed the same way whatever the stripe, so the
test isolates what the host adds: stripe bounds, the iteration order with the reference's
`Pts = nextPts` aliasing (similarity_fusion.py:157-177), the per-step all-gather of B and the
final gather. The kernels themselves are checked against scipy on the GPU
(test_gpu_plugin.py::test_snf_rows_split_bitexact, test_gpu_multirank.py)."""
import socket

import numpy as np
import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fake_lib(monkeypatch_like):
    """Install the CPU restatement of the two step halves (and of the whole step) into _lib."""
    import torch
    from acoss import _lib

    def diffuse_rows(stripes, skip, n, J, V, out=None, validated=False):
        others = [m for i, m in enumerate(stripes) if i != skip]
        A = others[0].clone()
        for m in others[1:]:
            A = A + m
        A = A / float(len(stripes) - 1)
        J, V = torch.as_tensor(J).long(), torch.as_tensor(V, dtype=torch.float64)
        B = torch.zeros_like(A)
        for k in range(J.shape[1]):  # B[a, j] += V[j, k] * A[a, J[j, k]], elementwise
            B = B + V[:, k][None, :] * A[:, J[:, k]]
        return B

    def left_rows(B, row0, rows, J, V, reg_diag, out=None, validated=False):
        J, V = torch.as_tensor(J).long(), torch.as_tensor(V, dtype=torch.float64)
        o = torch.zeros((rows, B.shape[1]), dtype=torch.float64)
        for k in range(J.shape[1]):
            o = o + V[row0:row0 + rows, k][:, None] * B[J[row0:row0 + rows, k]]
        if reg_diag > 0:
            idx = torch.arange(rows)
            o[idx, idx + row0] += reg_diag
        return o

    def step(mats, skip, J, V, reg_diag, out=None, validated=False):
        n = mats[0].shape[0]
        return left_rows(diffuse_rows(mats, skip, n, J, V), 0, n, J, V, reg_diag)

    monkeypatch_like(_lib, "_torch", lambda: torch)
    monkeypatch_like(_lib, "snf_diffuse_rows", diffuse_rows)
    monkeypatch_like(_lib, "snf_left_rows", left_rows)
    monkeypatch_like(_lib, "snf_step", step)


def _inputs(n, L, seed):
    rng = np.random.default_rng(seed)
    Ws = []
    for _ in range(L):
        D = rng.random((n, n))
        D = D + D.T
        Ws.append(np.exp(-D))
    return Ws


def _rank_worker(rank, world, port, n, L, K, niters, out, mode):
    import json
    import os
    import torch
    import torch.distributed as dist
    os.environ["ACOSS_SNF_SHARD"] = mode
    _fake_lib(setattr)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    from acoss.algorithms.utils import similarity_fusion as sf
    F = sf._fusion_ws([torch.as_tensor(W) for W in _inputs(n, L, 3)], K, niters, 1)
    np.save(out % rank, F.numpy())
    with open((out % rank) + ".plan.json", "w") as f:
        json.dump(sf.LAST_PLAN, f)
    dist.barrier()
    dist.destroy_process_group()


def _world(tmp_path, world, n, L, K, niters, mode):
    import json
    import torch.multiprocessing as mp
    out = str(tmp_path / ("%s_rank%%d.npy" % mode))
    mp.start_processes(_rank_worker, args=(world, _free_port(), n, L, K, niters, out, mode), nprocs=world,
                       join=True, start_method="spawn")
    res = [np.load(out % r) for r in range(world)]
    plans = [json.load(open((out % r) + ".plan.json")) for r in range(world)]
    return res, plans


@pytest.mark.parametrize("world,n,L", [(2, 37, 2), (3, 50, 3)])
def test_sharded_fusion_equals_world1(tmp_path, monkeypatch, world, n, L):
    """Forced sharding (ACOSS_SNF_SHARD=1), forced replication (=0) and the measured rule (auto)
    all give the world-1 result bit for bit; under auto every rank takes the same decision, from
    the same max-over-ranks timings."""
    import torch
    from acoss.algorithms.utils import similarity_fusion as sf
    _fake_lib(monkeypatch.setattr)
    K, niters = 5, 4
    ref = sf._fusion_ws([torch.as_tensor(W) for W in _inputs(n, L, 3)], K, niters, 1).numpy()
    assert np.isfinite(ref).all() and ref.shape == (n, n)
    for mode in ("1", "0", "auto"):
        res, plans = _world(tmp_path, world, n, L, K, niters, mode)
        for r in range(world):
            np.testing.assert_array_equal(res[r], ref)
        if mode == "0":
            assert plans == [{}] * world  # replicated: no plan measured
        else:
            assert all(p == plans[0] for p in plans), plans  # one decision, identical on every rank
            assert plans[0]["shard"] is (True if mode == "1" else plans[0]["rule_shard"])
            # forced sharding pays for no probe; auto measures both operations
            assert (plans[0]["t_step_replicated_ms"] is None) == (mode == "1")
            assert plans[0]["n"] == n and plans[0]["world"] == world


def test_shard_rows_cover():
    from acoss.algorithms.utils.similarity_fusion import shard_rows
    for n, w in [(10, 3), (15000, 8), (7, 7), (9, 2), (9, 8)]:
        b = shard_rows(n, w)
        assert b[0][0] == 0 and b[-1][1] == n and len(b) == w
        assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
        assert max(r1 - r0 for r0, r1 in b) - min(r1 - r0 for r0, r1 in b) <= 1
        assert all(r1 > r0 for r0, r1 in b)
