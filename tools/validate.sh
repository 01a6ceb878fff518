#!/bin/bash
# Validation of the tree on the GPU box: GPU tests, bench line, rocprof evidence.
#   bash tools/validate.sh <tag>      (through gpurun; then python tools/summarize_profile.py <tag> profiles/r01)
set -e
TAG=${1:?tag}
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
tail -2 gpurun_out/gputests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
timeout -k 10 1200 bash profiles/profile.sh $TAG > gpurun_out/prof.log 2>&1
echo ALLDONE
