#!/bin/bash
# CRP GPU tests on each named variant, then A/B timing: bash tools/ab1.sh <name>...
cd ${GRAFT_REPO_ROOT:-.}
for v in "$@"; do
  [ $v = base ] && continue
  echo "tests $v"
  ACOSS_HIP_LIB=$PWD/tools/abl/libabl_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_crp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1_$v.log 2>&1 || { tail -30 gpurun_out/ab1_$v.log; exit 1; }
  tail -1 gpurun_out/ab1_$v.log
done
bash tools/abrun.sh 13366 "$@" "$@"
