#!/bin/bash
# Stall-reason and instruction-cache counters of the bench workload (one stream), two rocprofv3
# --pmc passes: bash tools/pmc_stall.sh  ->  gpurun_out/pmcx/{a,b}/
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcx
mkdir -p "$OUT"
export TMPDIR=/tmp ACOSS_SPLIT_STREAMS=1
cd /tmp
B="$R/bench.py --steps 1 --warmup 1 --cpu-sample 0 --no-profile --no-paths"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM --output-format csv -d "$OUT/a" -o run -- python3 $B > "$OUT/a.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES --output-format csv -d "$OUT/b" -o run -- python3 $B > "$OUT/b.log" 2>&1
echo done
