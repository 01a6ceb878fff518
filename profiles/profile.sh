#!/bin/bash
# Collect the rocprofv3 evidence for one round (run on the GPU box through gpurun).
#   bash profiles/profile.sh <tag>
# 1) kernel trace + stats of a short bench run; 2) SQ instruction counters; 3) FETCH_SIZE and
# WRITE_SIZE in separate passes (TCC slots), per MI355X_MICROARCH.md §HBM / §rocprofv3.
set -euo pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --steps 1 --warmup 1 --cpu-sample 0 --no-profile"
timeout -k 10 300 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 $B > "$OUT/kt.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d "$OUT/sq" -o run -- python3 $B > "$OUT/sq.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $B > "$OUT/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $B > "$OUT/write.log" 2>&1
echo done
