#!/bin/bash
# SQ counters of the current build under env settings: bash tools/pmc_mode.sh <tag> "<ENV=..>" ...
cd ${GRAFT_REPO_ROOT:-.}
R=$PWD; TAG=$1; shift
export TMPDIR=/tmp ACOSS_SPLIT_STREAMS=1
i=0
for envs in "$@"; do
  i=$((i+1)); O=$R/gpurun_out/pmcd_${TAG}_$i
  echo "$envs" > $O.env
  env $envs timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU --output-format csv -d $O/a -o run -- python3 $R/tools/kbench.py --pairs 2000 --reps 1 --noprof > $O.a.log 2>&1 || exit 1
  env $envs timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_SCA --output-format csv -d $O/b -o run -- python3 $R/tools/kbench.py --pairs 2000 --reps 1 --noprof > $O.b.log 2>&1 || exit 1
done
echo pmc done
