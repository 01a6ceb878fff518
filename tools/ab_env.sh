#!/bin/bash
# A/B of the in-tree build under environment settings: bash tools/ab_env.sh "VAR=val ..." ...
cd ${GRAFT_REPO_ROOT:-.}
for spec in "$@"; do
  echo "env: $spec"
  env $spec timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 4 --noprof 2>&1 | grep -E "rep [23]|checksum" || exit 1
done
