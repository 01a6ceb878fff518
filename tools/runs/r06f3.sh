set -e
export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1
