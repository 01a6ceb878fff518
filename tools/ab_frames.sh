#!/bin/bash
# A/B of named variants at several track lengths: bash tools/ab_frames.sh "500 2000" base v1 v2 ...
cd ${GRAFT_REPO_ROOT:-.}
F=$1; shift
for f in $F; do
  for v in "$@"; do
    if [ $v = base ]; then L=acoss-1_amd/acoss/lib/libacoss_hip.so; else L=tools/abl/libabl_$v.so; fi
    echo "frames $f variant $v"
    ACOSS_HIP_LIB=$PWD/$L timeout -k 10 120 python tools/kbench.py --pairs 13366 --frames $f --reps 4 --noprof 2>&1 | grep -E "rep [23]|checksum" || exit 1
  done
done
