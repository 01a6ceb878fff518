"""One SiMPle call (every ordered pair of N tracks x F frames) for rocprofv3 passes.
    python tools/simple_one.py [F] [N] [MFMA 0|1]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "acoss-1_amd")]
from acoss import _lib  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
N = int(sys.argv[2]) if len(sys.argv) > 2 else 40
os.environ["ACOSS_SIMPLE_MFMA"] = sys.argv[3] if len(sys.argv) > 3 else "1"
rng = np.random.default_rng(7)
feats = []
for _ in range(N):
    X = np.abs(rng.standard_normal((12, F))) + 1e-3
    feats.append(X / np.linalg.norm(X, axis=0, keepdims=True))
pairs = np.array([(i, j) for i in range(N) for j in range(N) if i != j], np.int32)
flat = torch.as_tensor(np.concatenate([f.ravel() for f in feats])).cuda()
off = np.arange(N, dtype=np.int64) * 12 * F
lens = np.full(N, F, np.int32)
pt = torch.as_tensor(pairs).cuda()
for _ in range(2):
    s, _ = _lib.simple_mp_packed(flat, off, lens, pt)
torch.cuda.synchronize()
print("ok", float(s[0]))
