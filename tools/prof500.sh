#!/bin/bash
# One-stream kernel trace + SQ counters of one acoss_crp_align call at a given track length
# (kbench), for the per-line cost of the short-line selects.  bash tools/prof500.sh [frames] [tag]
set -euo pipefail
F=${1:-500}; TAG=${2:-p500}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp ACOSS_SPLIT_STREAMS=1
cd /tmp
B="$R/tools/kbench.py --frames $F --pairs 13366 --reps 2 --noprof"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 $B > "$OUT/kt.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d "$OUT/sq" -o run -- python3 $B > "$OUT/sq.log" 2>&1
echo done
