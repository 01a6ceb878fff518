"""Diagnostic: per-line event counts of the split selects (needs a -DACOSS_STAMPS build):
search passes, exact-key group recomputes and their sizes, le_bits recomputes, rows vs columns.
    bash tools/abbuild.sh stamps -DACOSS_STAMPS
    ACOSS_HIP_LIB=tools/abl/libabl_stamps.so python tools/select_counts.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "acoss-1_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from acoss import _lib  # noqa: E402
from acoss.engine import ChromaBank  # noqa: E402
from bench import corpus_tracks  # noqa: E402

lib = _lib.load_library()
tracks, _ = corpus_tracks(1, 2000, 20250101)
bank = ChromaBank(tracks)
T = len(tracks)
allp = np.array([(i, j) for i in range(T) for j in range(i + 1, T)], np.int32)
sel = np.random.default_rng(0).choice(len(allp), 2000, replace=False)
pairs = torch.as_tensor(allp[np.sort(sel)]).cuda()
out = (ctypes.c_ulonglong * 48)()
lib.acoss_debug_sweep_stamps(out)
bank.crp_align(pairs)
torch.cuda.synchronize()
lib.acoss_debug_sweep_stamps(out)
for name, b in (("rows", 6), ("cols", 11)):
    n = max(out[b], 1)
    print("%s: lines %d  passes/line %.2f  group recomputes/line %.3f  mean group %.2f  le_bits recomputes/line %.3f"
          % (name, out[b], out[b + 1] / n, out[b + 2] / n, out[b + 3] / max(out[b + 2], 1), out[b + 4] / n))
for name, b in (("rows", 16), ("cols", 18)):
    n = max(out[b], 1)
    print("%s unhinted: lines %d  passes/line %.2f" % (name, out[b], out[b + 1] / n))
h = [out[20 + k] for k in range(8)]
print("|P - hint| histogram (0,1,2,3-4,5-8,9-16,17-32,>32):", h, ["%.3f" % (x / max(sum(h), 1)) for x in h])
