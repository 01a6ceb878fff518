#!/bin/bash
# EarlyFusion A/B of environment settings on the in-tree library (tools/ef_bench.py pairs/s and
# score checksum per setting):  bash tools/ef_ab_env.sh "VAR=val ..." ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for e in "$@"; do
  echo "== [$e]"
  env $e timeout -k 10 120 python tools/ef_bench.py --reps 3 2>&1 | grep -v amdgpu.ids || exit 1
done
