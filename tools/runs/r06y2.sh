set -e
export TMPDIR=/tmp
O=gpurun_out/r06y2; mkdir -p $O
ACOSS_HIP_LIB=tools/abl/libabl_nopf.so timeout -k 10 300 python -u tools/simple_mfma_ab.py --out $O/nopf.json > $O/nopf.log 2>&1
timeout -k 10 300 python -u tools/simple_mfma_ab.py --out $O/pf.json > $O/pf.log 2>&1
ACOSS_HIP_LIB=tools/abl/libabl_nopf.so timeout -k 10 300 python -u tools/simple_mfma_ab.py --out $O/nopf2.json > $O/nopf2.log 2>&1
