set -e
export TMPDIR=/tmp
O=gpurun_out/r06z7; mkdir -p $O
for v in nomfma nofold; do ACOSS_HIP_LIB=tools/abl/libabl_$v.so timeout -k 10 300 python -u tools/simple_mfma_ab.py --out $O/$v.json > $O/$v.log 2>&1 || true; done
timeout -k 10 300 python -u tools/simple_mfma_ab.py --out $O/base.json > $O/base.log 2>&1
