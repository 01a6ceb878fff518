"""Basic-block summary of one kernel in a hipcc -S listing (instruction counts, memory / DPP /
ballot ops, branches): where the instructions of a select or sweep loop go.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude --cuda-device-only \
        -S -o /tmp/split.s acoss-1_amd/csrc/crp_split.hip
    python tools/isa_blocks.py /tmp/split.s k_sel_cols9 [min_instructions]
"""
import re
import sys
from collections import Counter

path, kname = sys.argv[1], sys.argv[2]
minn = int(sys.argv[3]) if len(sys.argv) > 3 else 0
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*%s\w*:" % kname, l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.section") or re.match(r"^_Z\w*:", lines[i]))
KINDS = ("ds_", "global_", "buffer_", "s_load", "v_readlane", "v_readfirstlane", "v_bcnt", "v_cmp", "v_pk_", "v_fma",
         "s_barrier", "s_waitcnt", "s_nop")
blocks, cur = [], None
for l in lines[start:end]:
    s = l.strip()
    m = re.match(r"^(\.LBB\d+_\d+):", s)
    if m:
        cur = [m.group(1), 0, Counter(), []]
        blocks.append(cur)
        continue
    if not s or s[0] in ";." or s.endswith(":"):
        continue
    if cur is None:
        cur = ["entry", 0, Counter(), []]
        blocks.append(cur)
    op = s.split()[0]
    cur[1] += 1
    if "dpp" in s:
        cur[2]["dpp"] += 1
    for k in KINDS:
        if op.startswith(k):
            cur[2][k] += 1
    if op.startswith("s_cbranch") or op == "s_branch":
        cur[3].append(s.split(";")[0].strip())
tot = sum(b[1] for b in blocks)
print("%s: %d instructions in %d blocks" % (kname, tot, len(blocks)))
for name, n, c, br in blocks:
    if n >= minn:
        print("%-14s %5d  %s  %s" % (name, n, dict(c), br))
