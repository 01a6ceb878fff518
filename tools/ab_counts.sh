#!/bin/bash
# select_counts for named stamps variants: bash tools/ab_counts.sh <name>...
cd ${GRAFT_REPO_ROOT:-.}
for v in "$@"; do
  echo "variant=$v"
  ACOSS_HIP_LIB=$PWD/tools/abl/libabl_$v.so timeout -k 10 120 python tools/select_counts.py || exit 1
done
