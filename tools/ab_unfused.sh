#!/bin/bash
cd ${GRAFT_REPO_ROOT:-.}
ACOSS_FUSE_ROWS=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_crp.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
for f in 0 1 0 1; do
  echo "fuse=$f"
  ACOSS_FUSE_ROWS=$f timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 --noprof 2>&1 | grep -E "rep 2|checksum"
  ACOSS_FUSE_ROWS=$f ACOSS_SPLIT_STREAMS=1 timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"
done
