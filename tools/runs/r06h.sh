set -e
export TMPDIR=/tmp
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 python -u tools/simple_mfma_ab.py --out $O/ovl.json > $O/ovl.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_misc.py tests/test_gpu_edges.py tests/test_gpu_plugin.py tests/test_gpu_multirank.py > $O/tests.txt 2>&1
