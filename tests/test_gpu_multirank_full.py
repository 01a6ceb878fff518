"""The multi-rank plugin flow at the Da-TACOS benchmark's full track count (configs 3 and 4's
8-GPU leg, rehearsed with 2 gloo ranks sharing one GPU): 15,000 songs in the benchmark
subset's clique structure (1,000 cliques x 13 + 2,000 singletons) through Serra09
(`downsample_fac=1`, 112.5 M unordered pairs) and SiMPle (crema, WIN=2, SKIP=1, 225 M ordered
pairs)
`all_pairwise` (algorithm_template.py:142-193): each rank scores its cost-balanced row stripe
on the device, the stripes are all-gathered and the matrix finished on the device. The assembled
Ds must equal the world-1 run bit for bit (SHA-256 of the whole 15,000 x 15,000 matrix, checked
by tests/multirank_worker.py with ACOSS_MR_DIGEST=1). Short tracks (the discriminative corpus at
a 48-frame base) keep the whole run to about a minute per world.
"""
import numpy as np
import pytest

from acoss import synthetic
from test_gpu_multirank import _run

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def datacos_full(tmp_path_factory):
    root = tmp_path_factory.mktemp("dtfull")
    tracks, labels = synthetic.make_hard_corpus("datacos", frames=48, seed=20250101, fixed_length=False)
    tracks, labels = tracks[:15000], np.asarray(labels[:15000], np.int32)
    assert len(tracks) == 15000
    csv, fdir = synthetic.write_feature_dataset(str(root), tracks, labels, chroma_keys=("hpcp", "crema"))
    return root, csv, fdir


@pytest.mark.timeout(900)
@pytest.mark.parametrize("algo", ["Serra09", "Simple"])
def test_world2_equals_world1_full_size(datacos_full, algo):
    root, csv, fdir = datacos_full
    env = {"ACOSS_MR_DIGEST": "1", "ACOSS_MR_DOWNSAMPLE": "1", "ACOSS_MR_SIMPLE_WIN": "2", "ACOSS_MR_SIMPLE_SKIP": "1"}
    d1 = _run(algo, 1, root, csv, fdir, "full", env_extra=env, timeout=600)
    d2 = _run(algo, 2, root, csv, fdir, "full", env_extra=env, timeout=600)
    assert set(d1) == set(d2) and d1
    for k in d1:
        assert d1[k][1] == str((15000, 15000)), d1[k]
        assert int(d1[k][2]) > 0
        assert d1[k][0] == d2[k][0], (k, d1[k], d2[k])


@pytest.fixture(scope="module")
def datacos_full_ef(tmp_path_factory):
    root = tmp_path_factory.mktemp("dtfull_ef")
    tracks, labels = synthetic.make_hard_corpus("datacos", frames=240, seed=20250101, fixed_length=False)
    tracks, labels = tracks[:15000], np.asarray(labels[:15000], np.int32)
    csv, fdir = synthetic.write_feature_dataset(str(root), tracks, labels, with_mfcc=True, beat_period=5,
                                                chroma_keys=("hpcp",), mfcc_from_chroma=True)
    return root, csv, fdir


@pytest.mark.timeout(900)
def test_earlyfusion_world2_equals_world1_full_size(datacos_full_ef):
    """Config 5 through coverid.benchmark("EarlyFusionTraile") at the Da-TACOS track count on one and
    on two gloo ranks: the four score matrices are all-gathered onto both ranks, the SNF late and
    early+late fusions run on both (sharded by the measured rule), and all six 15,000 x 15,000
    matrices have the world-1 SHA-256."""
    root, csv, fdir = datacos_full_ef
    env = {"ACOSS_MR_DIGEST": "1"}
    d1 = _run("bench:EarlyFusionTraile", 1, root, csv, fdir, "full", env_extra=env, timeout=800)
    d2 = _run("bench:EarlyFusionTraile", 2, root, csv, fdir, "full", env_extra=env, timeout=800)
    assert set(d1) == set(d2) == {"mfccs", "ssms", "chromas", "early", "late", "early+late"}
    for k in d1:
        assert d1[k][1] == str((15000, 15000)), d1[k]
        assert int(d1[k][2]) > 0
        assert d1[k][0] == d2[k][0], (k, d1[k], d2[k])
