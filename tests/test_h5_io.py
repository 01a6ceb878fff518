"""The HDF5 branches of the I/O (f4, CPU): '<prefix>_Ds.h5' written by CoverAlgorithm._save_Ds and
read back by _load_Ds (algorithm_template.py:163-166,193), and a deepdish-layout feature file
(datasets, a nested group, string attributes; extractors.py:114) read by features_io.load_features.

This image's python has no h5py, so the test runs those code paths in the other interpreter
that has one (/opt/conda/bin/python3.9 with h5py 3.3.0); it skips where
that interpreter is absent (e.g. on the GPU box). The product code is the same file in both."""
import os
import subprocess

import pytest

from conftest import ROOT

PY39 = "/opt/conda/bin/python3.9"

SCRIPT = r'''
import os, sys, numpy as np, h5py
sys.path.insert(0, os.path.join(sys.argv[1], "acoss-1_amd"))
from acoss import features_io
from acoss.algorithms.algorithm_template import CoverAlgorithm
tmp = sys.argv[2]
rng = np.random.default_rng(0)
# Ds persistence
a = CoverAlgorithm.__new__(CoverAlgorithm)
a.Ds = {"qmax": rng.random((7, 7)).astype(np.float32), "dmax": rng.random((7, 7)).astype(np.float32)}
prefix = os.path.join(tmp, "Chen_t")
a._save_Ds(prefix)
assert os.path.exists(prefix + "_Ds.h5") and os.path.exists(prefix + "_Ds.npz")
with h5py.File(prefix + "_Ds.h5", "r") as f:
    assert sorted(f.keys()) == ["dmax", "qmax"] and f["qmax"].dtype == np.float32
b = CoverAlgorithm.__new__(CoverAlgorithm)
os.remove(prefix + "_Ds.npz")          # the .h5 alone must be enough
b._load_Ds(prefix)
for k in a.Ds:
    assert np.array_equal(b.Ds[k], a.Ds[k]), k
# a deepdish-layout feature file: arrays as datasets, a nested dict as a group, strings as attrs
path = os.path.join(tmp, "W1", "T1.h5")
os.makedirs(os.path.dirname(path))
hpcp = rng.random((50, 12)).astype(np.float32)
with h5py.File(path, "w") as f:
    f.attrs["DEEPDISH_IO_VERSION"] = 12
    f.create_dataset("hpcp", data=hpcp, compression="gzip")
    f.create_dataset("mfcc_htk", data=rng.random((20, 50)).astype(np.float32))
    g = f.create_group("madmom_features")
    g.create_dataset("onsets", data=np.arange(0, 50, 7, dtype=np.int64))
    f.attrs["label"] = "W1"
    f.attrs["track_id"] = "T1"
d = features_io.load_features(path)
assert np.array_equal(d["hpcp"], hpcp) and d["label"] == "W1" and d["track_id"] == "T1"
assert np.array_equal(d["madmom_features"]["onsets"], np.arange(0, 50, 7))
# a blosc-compressed dataset (deepdish's default through PyTables) without the filter plugin:
# the chunk is stored as if blosc had been applied, so libhdf5 cannot read it; the reader must
# raise IOError naming blosc and the .npz conversion, not h5py's plugin-directory message
if not h5py.h5z.filter_avail(32001):
    bpath = os.path.join(tmp, "W1", "T2.h5")
    with h5py.File(bpath, "w") as f:
        ds = f.create_dataset("hpcp", shape=(50, 12), dtype="f4", chunks=(50, 12), compression=32001,
                              allow_unknown_filter=True)
        ds.id.write_direct_chunk((0, 0), hpcp.tobytes()[:1000], filter_mask=0)
        f.attrs["label"] = "W1"
    try:
        features_io.load_features(bpath)
        raise SystemExit("no error on a blosc dataset")
    except IOError as e:
        msg = str(e)
        assert "blosc" in msg and "save_features" in msg and "hpcp" in msg, msg
    # once converted (the .npz twin beside it), the same path reads
    features_io.save_features(bpath, {"hpcp": hpcp, "label": "W1"})
    assert np.array_equal(features_io.load_features(bpath)["hpcp"], hpcp)
print("OK")
'''


@pytest.mark.skipif(not os.path.exists(PY39), reason="no interpreter with h5py here")
def test_h5_paths_with_h5py(tmp_path):
    env = dict(os.environ)
    env.pop("PYTHONPATH", None)
    r = subprocess.run([PY39, "-c", SCRIPT, ROOT, str(tmp_path)], capture_output=True, text=True, env=env,
                       timeout=120)
    if r.returncode != 0 and "No module named 'h5py'" in r.stderr:
        pytest.skip("h5py not importable there")
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr
