"""Run the batched EarlyFusion on 80 synthetic 20000-frame tracks once (for rocprofv3)."""
import os, sys, tempfile, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "acoss-1_amd")]
import numpy as np
import torch
from acoss import synthetic
from acoss.algorithms.earlyfusion_traile import EarlyFusion
n = int(sys.argv[1]) if len(sys.argv) > 1 else 80
with tempfile.TemporaryDirectory() as tmp:
    tracks, labels = synthetic.make_corpus("covers80", frames=20000, seed=3, stretch=False)
    csv, fdir = synthetic.write_feature_dataset(tmp, tracks[:n], labels[:n], with_mfcc=True)
    ef = EarlyFusion(csv, fdir, shortname="p", cachedir=os.path.join(tmp, "cache"))
    ef.prepare()
    pairs = np.array([(i, j) for i in range(ef.N) for j in range(i + 1, ef.N)], np.int32)
    ef.similarity(pairs[:8]); torch.cuda.synchronize()
    t0 = time.perf_counter(); ef.similarity(pairs); torch.cuda.synchronize()
    print("pairs/s", len(pairs) / (time.perf_counter() - t0))
