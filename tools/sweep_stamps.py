"""Diagnostic: per-phase cycles of the fused sweep (k_sweep_rows9), per wave.
Needs a build with -DACOSS_STAMPS: bash tools/abbuild.sh stamps -DACOSS_STAMPS, then
ACOSS_HIP_LIB=tools/abl/libabl_stamps.so python tools/sweep_stamps.py"""
import ctypes, os, sys
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
pairs = torch.as_tensor(np.array([(i, j) for i in range(T) for j in range(i + 1, T)], np.int32)[:4000]).cuda()
out = (ctypes.c_ulonglong * 8)()
bank.crp_align(pairs); torch.cuda.synchronize(); lib.acoss_debug_sweep_stamps(out)
bank.crp_align(pairs); torch.cuda.synchronize(); lib.acoss_debug_sweep_stamps(out)
blocks = out[5]
names = ["fill+2 barriers", "diagonal walk", "barrier after walk", "Hc stores+barrier+roll", "row select"]
tot = sum(out[i] for i in range(5))
for i, nm in enumerate(names):
    print("%-24s %10.0f cycles/wave  %5.1f%%" % (nm, out[i] / blocks / 4, 100.0 * out[i] / tot))
print("blocks", blocks)
