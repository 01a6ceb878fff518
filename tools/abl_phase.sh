#!/bin/bash
# Per-phase HIP-event times of A/B variants: bash tools/abl_phase.sh <pairs> <name>...

cd ${GRAFT_REPO_ROOT:-.}
P=$1; shift
for v in "$@"; do
  if [ $v = base ]; then L=acoss-1_amd/acoss/lib/libacoss_hip.so; else L=tools/abl/libabl_$v.so; fi
  echo "variant=$v"
  ACOSS_HIP_LIB=$PWD/$L timeout -k 10 120 python tools/kbench.py --pairs $P --reps 3 --noprof 2>&1 | grep -E "rep 2|checksum"
  ACOSS_SPLIT_STREAMS=1 ACOSS_HIP_LIB=$PWD/$L timeout -k 10 120 python tools/kbench.py --pairs $P --reps 3 2>&1 | grep -E "rep 2"
done
