#!/bin/bash
cd ${GRAFT_REPO_ROOT:-.}
ACOSS_SWEEP=sys timeout -k 10 300 python -u -m pytest tests/test_gpu_crp.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
for m in sys valu sys valu; do
  echo "sweep=$m"
  ACOSS_SWEEP=$m timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 --noprof 2>&1 | grep -E "rep 2|checksum"
  ACOSS_SWEEP=$m ACOSS_SPLIT_STREAMS=1 timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"
done
