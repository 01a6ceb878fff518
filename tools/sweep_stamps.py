"""Diagnostic: per-phase s_memtime sums of the fused sweep (k_sweep_rows9) and the column
select (k_sel_cols9), per wave / per line.
Needs a build with -DACOSS_STAMPS: bash tools/abbuild.sh stamps -DACOSS_STAMPS, then
ACOSS_HIP_LIB=tools/abl/libabl_stamps.so python tools/sweep_stamps.py [frames]"""
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

FRAMES = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
lib = _lib.load_library()
tracks, _ = corpus_tracks(1, FRAMES, 20250101)
bank = ChromaBank(tracks)
T = len(tracks)
pairs = torch.as_tensor(np.array([(i, j) for i in range(T) for j in range(i + 1, T)], np.int32)[:4000]).cuda()
out = (ctypes.c_ulonglong * 48)()
bank.crp_align(pairs)
torch.cuda.synchronize()
lib.acoss_debug_sweep_stamps(out)
bank.crp_align(pairs)
torch.cuda.synchronize()
lib.acoss_debug_sweep_stamps(out)
blocks = out[5]
rows = blocks * 32
names = ["fill / norms+Gram", "walk (VALU) / barrier", "barrier / walk (MFMA)", "Hc stores+barrier+roll", "row select"]
tot = sum(out[i] for i in range(5))
print("mode", os.environ.get("ACOSS_SWEEP", "mfma"), "blocks", blocks)
for i, nm in enumerate(names):
    print("%-28s %10.0f per wave  %5.1f%%" % (nm, out[i] / blocks / 4, 100.0 * out[i] / tot))
cols = max(out[31], 1)
print("column select per column: search %.0f  group %.0f  threshold %.0f  le_bits+word %.0f  (%d columns)"
      % (out[32] / cols, out[33] / cols, out[34] / cols, out[35] / cols, cols))
print("row select per row: search %.0f  group %.0f  threshold %.0f" % (out[36] / rows, out[37] / rows, out[38] / rows))
for side, (ln, ps, gr, mem, leg, uh, uhp) in (("rows", (6, 7, 8, 9, 10, 16, 17)), ("cols", (11, 12, 13, 14, 15, 18, 19))):
    n = max(out[ln], 1)
    print("%s: lines %d  passes/line %.2f  group rounds/line %.2f  members/group %.2f  le-group recomputes/line %.3f  "
          "unhinted %.3f (passes %.2f)" % (side, out[ln], out[ps] / n, out[gr] / n, out[mem] / max(out[gr], 1),
                                           out[leg] / n, out[uh] / n, out[uhp] / max(out[uh], 1)))
print("hint distance histogram (0,1,2,<=4,<=8,<=16,<=32,>32):", [int(out[20 + b]) for b in range(8)])
