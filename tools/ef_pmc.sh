#!/bin/bash
# SQ counters of the EarlyFusion kernels (tools/ef_bench.py, one repetition), two passes.
#   bash tools/ef_pmc.sh <tag> [lib]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; LIB=${2:-acoss-1_amd/acoss/lib/libacoss_hip.so}
OUT=$R/gpurun_out/efpmc_$TAG; mkdir -p $OUT
export TMPDIR=/tmp ACOSS_HIP_LIB=$R/$LIB
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/a -o run -- python3 $R/tools/ef_bench.py --reps 1 > $OUT/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD --output-format csv -d $OUT/b -o run -- python3 $R/tools/ef_bench.py --reps 1 > $OUT/b.log 2>&1
echo efpmc-done
