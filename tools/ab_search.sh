#!/bin/bash
# secant vs gallop search: correctness, pass counts, speed
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 300 python -u -m pytest tests/test_gpu_crp.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
for v in stamps stamps_old; do echo "== $v"; ACOSS_HIP_LIB=$PWD/tools/abl/libabl_$v.so timeout -k 10 120 python tools/select_counts.py 2>&1 | tail -4; done
bash tools/abrun.sh 13366 base gallop base gallop
