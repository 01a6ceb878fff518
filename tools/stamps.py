"""Diagnostic: per-phase cycle shares of k_crp_select16 (needs ACOSS_DEBUG_STAMPS=1)."""
import ctypes, os, sys
os.environ["ACOSS_DEBUG_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "acoss-1_amd")]
import numpy as np, torch
from acoss import _lib
from acoss.engine import ChromaBank
from bench import corpus_tracks
lib = _lib.load_library()
tracks, _ = corpus_tracks(1, 2000, 20250101)
bank = ChromaBank(tracks)
T = len(tracks)
pairs = torch.as_tensor(np.array([(i, j) for i in range(T) for j in range(i + 1, T)], np.int32)[:2000]).cuda()
out = (ctypes.c_ulonglong * 8)()
bank.crp_align(pairs); torch.cuda.synchronize(); lib.acoss_debug_stamps(out)
bank.crp_align(pairs); torch.cuda.synchronize(); lib.acoss_debug_stamps(out)
n = out[4]
names = ["sweep", "phaseA(prefix)", "phaseB(exact keys)", "phaseC(rank+thr)"]
tot = sum(out[i] for i in range(4))
for i, nm in enumerate(names):
    print("%-20s %10.0f cycles/block  %5.1f%%" % (nm, out[i] / n, 100.0 * out[i] / tot))
print("blocks", n)
