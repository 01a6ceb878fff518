#!/bin/bash
# short-line selects: CRP parity on the variant, then A/B at 500 / 1000 / 2000 frames
cd ${GRAFT_REPO_ROOT:-.}
L=$PWD/tools/abl/libabl_${1:-short}.so
ACOSS_HIP_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_crp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_short.log 2>&1 || { tail -40 gpurun_out/ab_short.log; exit 1; }
tail -1 gpurun_out/ab_short.log
for f in 500 1000 2000; do
  for v in base short; do
    if [ $v = base ]; then E="ACOSS_NO_SHORT=1"; else E="ACOSS_X=1"; fi
    echo "frames $f $v"
    env $E ACOSS_HIP_LIB=$L timeout -k 10 120 python tools/kbench.py --pairs 13366 --frames $f --reps 4 --noprof 2>&1 | grep -E "rep [23]|checksum" || exit 1
  done
done
