#!/bin/bash
# correctness of the current build (CRP GPU tests) + A/B speed vs named variants
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 300 python -u -m pytest tests/test_gpu_crp.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
bash tools/abrun.sh 13366 "$@"
