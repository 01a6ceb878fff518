#!/bin/bash
# Round-1 validation of HEAD: GPU tests, bench line, rocprof evidence.
set -e
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 1200 bash profiles/profile.sh r01g > gpurun_out/prof.log 2>&1
echo ALLDONE
