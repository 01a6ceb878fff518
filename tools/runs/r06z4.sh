set -e
export TMPDIR=/tmp
O=gpurun_out/r06z4; mkdir -p $O
B="tools/bench_datacos.py --algo earlyfusion --frames 47 --blocks-lo 14 --max-pairs 1000000"
run() { ACOSS_EF_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$1 -o run -- python3 -u $B > $O/$1.log 2>&1; }
ACOSS_EF_PACK=0 run nopack
ACOSS_HIP_LIB=tools/abl/libabl_pk16.so run pk16
ACOSS_HIP_LIB=tools/abl/libabl_pk32.so run pk32
ACOSS_HIP_LIB=tools/abl/libabl_pk64.so run pk64
for v in pk16 pk32 pk64; do ACOSS_HIP_LIB=tools/abl/libabl_$v.so timeout -k 10 200 python -u $B > $O/wall_$v.log 2>&1; done
ACOSS_EF_PACK=0 timeout -k 10 200 python -u $B > $O/wall_nopack.log 2>&1
