set -e
export TMPDIR=/tmp
O=gpurun_out/r06z8; mkdir -p $O
timeout -k 10 300 python -u tools/simple_mfma_ab.py --out $O/ovl.json > $O/ovl.log 2>&1
