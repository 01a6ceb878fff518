#!/bin/bash
# Time A/B variants on the GPU box: bash tools/abrun.sh <pairs> <name>... ("base" = the in-tree build)
set -e
cd ${GRAFT_REPO_ROOT:-.}
P=$1; shift
for v in "$@"; do
  if [ $v = base ]; then L=acoss-1_amd/acoss/lib/libacoss_hip.so; else L=tools/abl/libabl_$v.so; fi
  echo "variant=$v"; ACOSS_HIP_LIB=$PWD/$L timeout -k 10 120 python tools/kbench.py --pairs $P --reps 4 --noprof 2>&1 | grep -E "rep [123]|checksum"
done
