#!/bin/bash
# EarlyFusion A/B on the GPU box: tools/ef_bench.py pairs/s and score checksum per library
# variant (base = the in-tree library; NAME = tools/abl/libabl_NAME.so from tools/abbuild.sh),
# plus ACOSS_EF_LDS_CSM=1 (the LDS-tiled CSM kernel) on the base library.
#   bash tools/ef_ab.sh VARIANT...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
echo "== base, ACOSS_EF_LDS_CSM=1"
ACOSS_EF_LDS_CSM=1 timeout -k 10 120 python tools/ef_bench.py --reps 3 2>&1 | grep -v amdgpu.ids || exit 1
for v in "$@"; do
  if [ "$v" = base ]; then L=$R/acoss-1_amd/acoss/lib/libacoss_hip.so; else L=$R/tools/abl/libabl_$v.so; fi
  echo "== $v"
  ACOSS_HIP_LIB=$L timeout -k 10 120 python tools/ef_bench.py --reps 3 2>&1 | grep -v amdgpu.ids || exit 1
done
