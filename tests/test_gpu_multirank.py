"""The real HIP scorers under torch.distributed: 2 gloo ranks sharing one GPU each score a
row stripe of a Da-TACOS-shaped mini corpus (13-song cliques plus singletons, ragged
lengths) through Serra09 / ChenFusion / Simple / EarlyFusion.all_pairwise
(algorithm_template.py:142-193), all-gather, symmetrise on the device; the assembled Ds must
equal the world-1 run bit for bit. ChenFusion's and EarlyFusion's SNF late fusions run
row-sharded (and, for EarlyFusion, replicated) across the same two ranks.
Ranks are child processes (subprocess), one GPU context each (3 with the parent)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from acoss import synthetic
from conftest import ROOT

pytestmark = pytest.mark.gpu

WORKER = os.path.join(ROOT, "tests", "multirank_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def datacos_mini(tmp_path_factory):
    root = tmp_path_factory.mktemp("dtmini")
    rng = np.random.Generator(np.random.PCG64(77))
    tracks, labels = [], []
    sizes = [13, 13, 13] + [1] * 9
    for lab, size in enumerate(sizes):
        base = synthetic.base_sequence(rng, int(rng.integers(200, 700)) * 40)
        for v in range(size):
            seq = base if v == 0 else synthetic.cover_of(rng, base)
            tracks.append(synthetic.render(rng, seq))
            labels.append(lab)
    csv, fdir = synthetic.write_feature_dataset(str(root), tracks, np.asarray(labels), with_mfcc=True)
    return root, csv, fdir


def _run(algo, world, root, csv, fdir, tag, env_extra=None, timeout=240):
    out = str(root / ("%s_%s_w%d.npz" % (algo, tag, world)))
    cache = str(root / ("cache_%s_%s_w%d" % (algo, tag, world)))
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0", **(env_extra or {}))
        procs.append(subprocess.Popen([sys.executable, WORKER, algo, csv, fdir, cache, out], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace"))
    for p, lg in zip(procs, logs):
        assert p.returncode == 0, lg[-3000:]
    with np.load(out) as z:
        return {k: np.array(z[k]) for k in z.files}


@pytest.mark.parametrize("algo", ["Serra09", "ChenFusion", "Simple"])
def test_world2_equals_world1(datacos_mini, algo):
    root, csv, fdir = datacos_mini
    d1 = _run(algo, 1, root, csv, fdir, "a")
    d2 = _run(algo, 2, root, csv, fdir, "b")
    assert set(d1) == set(d2)
    for k in d1:
        assert d1[k].shape == (48, 48)
        assert np.count_nonzero(d1[k]) > 48 * 30
        np.testing.assert_array_equal(d2[k], d1[k])


def test_late_fusion_sharded_equals_world1(datacos_mini):
    """ChenFusion's SNF late fusion (20 cross-diffusion steps per matrix) row-sharded over two
    ranks — one all-gather of B per step (similarity_fusion._fusion_sharded) — equals the
    single-process fusion bit for bit."""
    root, csv, fdir = datacos_mini
    d1 = _run("ChenLate", 1, root, csv, fdir, "a")
    d2 = _run("ChenLate", 2, root, csv, fdir, "b", {"ACOSS_SNF_SHARD": "1"})
    assert set(d1) == set(d2) and "Late" in d1
    assert np.count_nonzero(d1["Late"]) > 48 * 30
    for k in d1:
        np.testing.assert_array_equal(d2[k], d1[k])


@pytest.mark.parametrize("shard", ["1", "0"])
def test_earlyfusion_world2_equals_world1(datacos_mini, shard):
    """EarlyFusion (config 5) across two ranks: each scores its block-count-balanced stripe with
    the batched HIP scorer (_device_scores), the four score matrices are all-gathered, and the
    SNF late / early+late fusions run row-sharded (shard=1) or replicated on every rank (0): all
    six matrices equal the world-1 run bit for bit."""
    root, csv, fdir = datacos_mini
    d1 = _run("EarlyFusion", 1, root, csv, fdir, "a")
    d2 = _run("EarlyFusion", 2, root, csv, fdir, "b" + shard, {"ACOSS_SNF_SHARD": shard})
    assert set(d1) == set(d2) == {"mfccs", "ssms", "chromas", "early", "late", "early+late"}
    for k in d1:
        assert d1[k].shape == (48, 48)
        assert np.count_nonzero(d1[k]) > 48 * 30, k
        np.testing.assert_array_equal(d2[k], d1[k], err_msg=k)


@pytest.mark.parametrize("name", ["Serra09", "LateFusionChen"])
def test_benchmark_entry_point_world2(datacos_mini, name):
    """coverid.benchmark (coverid.py:22-148) on two gloo ranks sharing the GPU:
    Serra09 gathers Ds onto rank 0 only, LateFusionChen all-gathers it for the row-sharded SNF;
    either way the matrices equal the world-1 run bit for bit, rank 0 alone writes the results
    CSV (exactly one row per similarity type, the same rows as world 1), and no rank leaves a
    memmap file in the cache directory."""
    root, csv, fdir = datacos_mini
    algo = "bench:" + name
    d1 = _run(algo, 1, root, csv, fdir, "a")
    d2 = _run(algo, 2, root, csv, fdir, "b", {"ACOSS_SNF_SHARD": "1"})
    assert set(d1) == set(d2) and d1
    for k in d1:
        np.testing.assert_array_equal(d2[k], d1[k], err_msg=k)
    rows = {}
    for tag, world in (("a", 1), ("b", 2)):
        cache = root / ("cache_%s_%s_w%d" % (algo, tag, world))
        lines = (cache / ("results_mr_%s.csv" % name)).read_text().strip().splitlines()
        assert lines[0].startswith("name,")
        rows[world] = sorted(lines[1:])
        assert sorted(r.split(",")[0] for r in rows[world]) == sorted("%s_%s" % (name, k) for k in d1), lines
        assert not [f for f in os.listdir(cache) if "_dmat" in f], os.listdir(cache)
    assert rows[1] == rows[2]
