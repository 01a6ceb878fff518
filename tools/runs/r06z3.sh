set -e
export TMPDIR=/tmp
O=gpurun_out/r06z3; mkdir -p $O
B="tools/bench_datacos.py --algo earlyfusion --frames 47 --blocks-lo 14 --max-pairs 1000000"
run() { ACOSS_EF_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$1 -o run -- python3 -u $B > $O/$1.log 2>&1; }
ACOSS_EF_PACK=0 run nopack
run pack8
ACOSS_HIP_LIB=tools/abl/libabl_ord1.so run ord1
ACOSS_HIP_LIB=tools/abl/libabl_pk4.so run pk4
ACOSS_HIP_LIB=tools/abl/libabl_pk16.so run pk16
ACOSS_EF_PACK=0 run nopack_b
