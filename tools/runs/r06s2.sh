set -e
export TMPDIR=/tmp
O=gpurun_out/r06s2; mkdir -p $O
ACOSS_EF_PACK=0 timeout -k 10 100 python -u tools/ef_pack_debug.py $O/p0.npy > $O/p0.log 2>&1
ACOSS_EF_PACK=0 ACOSS_EF_STREAMS=1 timeout -k 10 100 python -u tools/ef_pack_debug.py $O/p0s.npy $O/p0.npy > $O/p0s.log 2>&1
ACOSS_EF_PACK=2 timeout -k 10 100 python -u tools/ef_pack_debug.py $O/p2.npy $O/p0.npy > $O/p2.log 2>&1
ACOSS_EF_PACK=1 timeout -k 10 100 python -u tools/ef_pack_debug.py $O/p1.npy $O/p0.npy > $O/p1.log 2>&1
ACOSS_EF_PACK=2 ACOSS_EF_STREAMS=1 timeout -k 10 100 python -u tools/ef_pack_debug.py $O/p2s.npy $O/p0.npy > $O/p2s.log 2>&1
