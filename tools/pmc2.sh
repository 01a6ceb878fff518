#!/bin/bash
# Two SQ counter passes (issue/wait breakdown) over one kbench call on ONE stream.
#   bash tools/pmc2.sh <tag> [lib]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; LIB=${2:-acoss-1_amd/acoss/lib/libacoss_hip.so}
OUT=$R/gpurun_out/pmc_$TAG; mkdir -p $OUT
export TMPDIR=/tmp ACOSS_SPLIT_STREAMS=1 ACOSS_HIP_LIB=$R/$LIB
cd /tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $OUT/a -o run -- python3 $R/tools/kbench.py --pairs 4000 --reps 1 --noprof > $OUT/a.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $OUT/b -o run -- python3 $R/tools/kbench.py --pairs 4000 --reps 1 --noprof > $OUT/b.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS SQ_CYCLES --output-format csv -d $OUT/c -o run -- python3 $R/tools/kbench.py --pairs 4000 --reps 1 --noprof > $OUT/c.log 2>&1
echo pmc-done
