"""bench.py's multi-rank launch contract (CPU): `--gpus N` must never silently measure fewer ranks.

* WORLD_SIZE set by a launcher but different from --gpus: bench.py refuses, before touching torch.
* --gpus N without a launcher: bench.py starts N rank processes itself (launch_ranks); when a rank
  fails (here: no GPU in this container) the parent stops the others and exits non-zero.
"""
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra, timeout=240):
    env = dict(os.environ, **env_extra)
    for k in ("RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    if "WORLD_SIZE" not in env_extra:
        env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


def test_world_size_mismatch_fails_loudly():
    r = _run(["--gpus", "8", "--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "1"})
    assert r.returncode != 0
    assert "--gpus 8 but WORLD_SIZE=1" in r.stderr
    assert r.stdout.strip() == ""  # no JSON line for a run that did not happen


def test_self_launch_propagates_rank_failure():
    # two ranks, no GPU here: every rank fails at its first GPU call; the parent must report it
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-paths", "--cpu-sample", "0"],
             {"ACOSS_DIST_BACKEND": "gloo"})
    assert r.returncode != 0, r.stderr[-2000:]
    assert r.stdout.strip() == ""


def test_launch_ranks_env(tmp_path, monkeypatch):
    """launch_ranks gives rank r the torch.distributed.run environment (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR 127.0.0.1, one MASTER_PORT) and relays only rank 0's JSON line (the
    process group's own stdout chatter goes to stderr)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    script = tmp_path / "rank.py"
    script.write_text("import os, json\nprint('[Gloo] Rank 0 is connected to 2 peer ranks.')\n"
                      "print(json.dumps({k: os.environ[k] for k in ('RANK', 'LOCAL_RANK', "
                      "'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT', 'ACOSS_BENCH_LAUNCHER')}))\n")
    import io
    buf = io.StringIO()
    monkeypatch.setattr(sys, "stdout", buf)
    assert bench.launch_ranks(3, script=str(script), argv=[]) == 0
    import json
    lines = [ln for ln in buf.getvalue().splitlines() if ln.strip()]
    assert len(lines) == 1
    env0 = json.loads(lines[0])
    assert env0["RANK"] == "0" and env0["LOCAL_RANK"] == "0" and env0["WORLD_SIZE"] == "3"
    assert env0["MASTER_ADDR"] == "127.0.0.1" and int(env0["MASTER_PORT"]) > 0
    assert env0["ACOSS_BENCH_LAUNCHER"] == "self"


def _diag_worker(rank, world, port, out):
    import json
    import numpy as np
    import torch.distributed as dist
    sys.path[:0] = [ROOT, os.path.join(ROOT, "acoss-1_amd")]
    import bench
    from acoss import distributed
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    lens = np.array([2000 - 7 * (i % 5) for i in range(40)], np.int32)
    bounds = distributed.stripe_bounds(lens, world, symmetric=True)
    d = bench.exchange_diagnostics(world, rank, 10.0 + rank, 2.0 + 0.5 * rank, 1.5, bounds, lens, len(lens), "cpu")
    if rank == 0:
        with open(out, "w") as f:
            json.dump(d, f)
    else:
        assert d is None
    dist.destroy_process_group()


def test_exchange_diagnostics_world2(tmp_path):
    """The per-rank fields a multi-GPU bench line carries, assembled on rank 0 over a
    gloo world of 2: compute / exchange ms per rank, the stripe's share of sum M'N', the imbalance
    and the all-gather's bandwidth."""
    import json
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "diag.json")
    mp.start_processes(_diag_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    d = json.load(open(out))
    assert [r["rank"] for r in d["per_rank"]] == [0, 1]
    for r in d["per_rank"]:
        assert set(r) >= {"rows", "pairs", "cost_share", "compute_ms_per_step", "exchange_ms_per_step",
                          "allgather_probe_ms"}
    assert abs(sum(r["cost_share"] for r in d["per_rank"]) - 1.0) < 1e-6
    assert sum(r["pairs"] for r in d["per_rank"]) == 40 * 39 // 2
    assert d["per_rank"][1]["compute_ms_per_step"] == 11.0 and d["per_rank"][1]["exchange_ms_per_step"] == 2.5
    assert d["imbalance"]["compute_max_over_min"] == round(11.0 / 10.0, 4)
    assert 1.0 <= d["imbalance"]["cost_max_over_min"] < 1.2
    ag = d["allgather"]
    assert ag["bytes_received_per_rank"] == ag["padded_rows"] * 40 * 4 and ag["gbps_per_rank"] is not None
