"""Compare EarlyFusion scores of one process against a saved .npy (ACOSS_EF_PACK variants) and
print the pairs that differ.   python tools/ef_pack_debug.py OUT.npy [REF.npy]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "acoss-1_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from acoss import _lib  # noqa: E402

rng = np.random.default_rng(5)
NT = 24
nb = rng.integers(40, 91, NT).astype(np.int32)
off = np.concatenate([[0], np.cumsum(nb[:-1])]).astype(np.int64)
R = int(nb.sum())
bank = {"mfccs": torch.as_tensor(rng.standard_normal((R, 1000), dtype=np.float32)).cuda(),
        "ssms": torch.as_tensor(np.abs(rng.standard_normal((R, 1225), dtype=np.float32))).cuda(),
        "chromas": torch.as_tensor(np.abs(rng.standard_normal((R, 480), dtype=np.float32))).cuda(),
        "chroma_med": torch.as_tensor(np.abs(rng.standard_normal((NT, 12), dtype=np.float32))).cuda(),
        "off": torch.as_tensor(off).cuda(), "nb": torch.as_tensor(nb).cuda(), "max_blocks": int(nb.max())}
pairs = np.array([(i, j) for i in range(NT) for j in range(i + 1, NT)], np.int32)
out = _lib.earlyfusion(bank, pairs, 0.1, 10).cpu().numpy()
np.save(sys.argv[1], out)
if len(sys.argv) > 2:
    ref = np.load(sys.argv[2])
    bad = np.flatnonzero((out != ref).any(1))
    print("differing pairs:", len(bad), [(int(b), tuple(pairs[b]), out[b].tolist(), ref[b].tolist()) for b in bad[:10]])
