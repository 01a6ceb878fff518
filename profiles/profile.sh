#!/bin/bash
# Collect the rocprofv3 evidence for one round (run on the GPU box through gpurun).
#   bash profiles/profile.sh <tag>
# Every pass runs the bench workload (2 acoss_crp_align calls: 1 warmup + 1 step) on ONE stream
# (ACOSS_SPLIT_STREAMS=1), so each kernel's durations add up to the call time:
# 1) kernel trace + stats; 2) SQ instruction counters; 3) FETCH_SIZE and 4) WRITE_SIZE in
# separate passes (TCC slots), per MI355X_MICROARCH.md §HBM / §rocprofv3.
set -euo pipefail
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp ACOSS_SPLIT_STREAMS=1
cd /tmp
B="$R/bench.py --steps 1 --warmup 1 --cpu-sample 0 --no-profile --no-paths"
# the build these counters belong to (bench.py refuses figures of another build)
python3 -c "import sys, json; sys.path.insert(0, '$R'); import bench; json.dump(bench.build_id(), open('$OUT/build.json', 'w'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 $B > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d "$OUT/sq" -o run -- python3 $B > "$OUT/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $B > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $B > "$OUT/write.log" 2>&1
echo done
