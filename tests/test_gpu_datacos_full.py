"""Configs 3 and 4 at the Da-TACOS benchmark's full track count, through the plugin API, on one GPU.

15,000 songs in the benchmark subset's clique structure (1,000 cliques x 13 + 2,000 singletons,
`acoss/data/da-tacos_benchmark_subset.csv`), written as per-song feature files in the reference's
layout and run through the reference flow (`coverid.py:57-70,124-139`): Serra09
`all_pairwise(symmetric=True)` -> `normalize_by_length` -> `getEvalStatistics` (112.5 M unordered
pairs) and SiMPle `all_pairwise(symmetric=False)` -> `getEvalStatistics` (225.0 M ordered pairs).

Tracks are short (the discriminative corpus at a 48-frame base, 34-67 frames) so the whole job
fits a test; every size-dependent part of the path runs at full size: the 1 M-pair chunk loop, the
15,000 x 15,000 Ds memmap and its device finish, the device evaluation. Checked
(tools/datacos_plugin.py): Ds symmetric with a zero diagonal and finite (Serra09) / finite off the
diagonal (SiMPle); a seeded uniform sample of 3,000 pairs == the CPU oracle; device MAP / MR1 /
MRR / MDR / Top-k == the host restatement of getEvalStatistics on the same matrix. The full-length
runs (500-frame base) are tools/datacos_plugin.py's, logged under profiles/r04/.

Config 5 (EarlyFusionTraile, coverid.py:72-88) at the same track count: per-song hpcp, mfcc_htk (43
frames shorter) and onset files; prepare() (beat-block features of all 15,000 songs on the GPU,
cached per song) -> all_pairwise (112.5 M pairs, four score matrices) -> do_late_fusion (SNF over 3
and over 4 matrices of 15,000 x 15,000) -> getEvalStatistics on all six keys. Checked: the four score
matrices symmetric / zero diagonal / finite; the block features of sampled songs == the numpy
restatement (1e-5); 3,000 sampled pairs' mfccs / ssms / chromas scores == the canonical-order CPU
oracle (oracle/ef_oracle.cpp); late / early+late finite; device statistics == host on two keys.
"""
import importlib.util
import os

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _tool():
    spec = importlib.util.spec_from_file_location("datacos_plugin", os.path.join(ROOT, "tools", "datacos_plugin.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.timeout(600)
@pytest.mark.parametrize("algo", ["serra09", "simple"])
def test_datacos_full_track_count(algo, tmp_path):
    tool = _tool()
    a = tool.parse_args(["--algo", algo, "--frames", "48", "--sample", "3000", "--threads", "8",
                         "--workdir", str(tmp_path)])
    res = tool.run(a)
    print(res)
    assert res["pairs"] == (112492500 if algo == "serra09" else 224985000)
    assert res["checks"]["sample_pairs"] == 3000
    assert res["checks"]["sample_pairs_differing_from_oracle"] == 0, res["checks"]
    assert all(v for v in res["checks"].values() if isinstance(v, bool)), res["checks"]
    assert res["ok"]
    assert 0.0 < res["MAP"] <= 1.0


@pytest.mark.timeout(600)
def test_datacos_full_track_count_earlyfusion(tmp_path):
    tool = _tool()
    a = tool.parse_args(["--algo", "earlyfusion", "--frames", "240", "--beat-period", "5", "--sample", "3000",
                         "--threads", "8", "--host-eval-keys", "early+late,chromas", "--workdir", str(tmp_path)])
    res = tool.run(a)
    print({k: v for k, v in res.items() if k != "stats"})
    assert res["pairs"] == 112492500
    assert res["checks"]["sample_pairs"] == 3000
    assert res["checks"]["sample_pairs_differing_from_oracle"] == 0, res["checks"]
    assert all(v for v in res["checks"].values() if isinstance(v, bool)), res["checks"]
    assert set(res["stats"]) == {"mfccs", "ssms", "chromas", "early", "late", "early+late"}
    assert res["ok"]
    assert 0.0 < res["stats"]["early+late"]["MAP"] <= 1.0
