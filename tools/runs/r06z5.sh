set -e
export TMPDIR=/tmp
O=gpurun_out/r06z5; mkdir -p $O
ACOSS_HIP_LIB=tools/abl/libabl_km1.so timeout -k 10 300 python -u tools/simple_mfma_ab.py --out $O/km1.json > $O/km1.log 2>&1
timeout -k 10 300 python -u tools/simple_mfma_ab.py --out $O/km2.json > $O/km2.log 2>&1
