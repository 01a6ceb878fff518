#!/bin/bash
# Round validation on the GPU box: GPU tests, smoke, default bench, then the rocprofv3 passes.
#   bash tools/validate.sh <tag>
set -euo pipefail
TAG=${1:-r01}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1
tail -3 gpurun_out/gputests_$TAG.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
cat gpurun_out/bench_$TAG.json
bash profiles/profile.sh "$TAG"
