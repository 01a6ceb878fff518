#!/bin/bash
# A/B of named variants on a mixed-length corpus: bash tools/ab_mixed.sh LO,HI v1 v2 ...
cd ${GRAFT_REPO_ROOT:-.}
R=$1; shift
HI=${R#*,}
for v in "$@"; do
  if [ $v = base ]; then L=acoss-1_amd/acoss/lib/libacoss_hip.so; else L=tools/abl/libabl_$v.so; fi
  echo "mixed $R variant $v"
  ACOSS_HIP_LIB=$PWD/$L timeout -k 10 120 python tools/kbench.py --pairs 13366 --frames $HI --mixed $R --reps 4 --noprof 2>&1 | grep -E "rep [23]|checksum" || exit 1
done
