#!/bin/bash
# Two SQ counter passes over kbench for a list of variants: bash tools/pmc_detail.sh <tag> <variant>...
cd ${GRAFT_REPO_ROOT:-.}
R=$PWD; TAG=$1; shift
export TMPDIR=/tmp
for v in "$@"; do
  if [ $v = base ]; then L=$R/acoss-1_amd/acoss/lib/libacoss_hip.so; else L=$R/tools/abl/libabl_$v.so; fi
  export ACOSS_HIP_LIB=$L ACOSS_SPLIT_STREAMS=1
  O=$R/gpurun_out/pmcd_${TAG}_$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU --output-format csv -d $O/a -o run -- python3 $R/tools/kbench.py --pairs 2000 --reps 1 --noprof > $O.a.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA --output-format csv -d $O/b -o run -- python3 $R/tools/kbench.py --pairs 2000 --reps 1 --noprof > $O.b.log 2>&1 || exit 1
done
echo pmc done
