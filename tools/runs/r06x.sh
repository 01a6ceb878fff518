set -e
export TMPDIR=/tmp
O=gpurun_out/r06x; mkdir -p $O
B="tools/bench_datacos.py --algo earlyfusion --frames 47 --blocks-lo 14 --max-pairs 4000000"
timeout -k 10 240 python -u $B > $O/rag_new.log 2>&1
ACOSS_HIP_LIB=tools/abl/libabl_r06v.so timeout -k 10 240 python -u $B > $O/rag_old.log 2>&1
ACOSS_EF_W4=0 timeout -k 10 240 python -u $B > $O/rag_w1.log 2>&1
ACOSS_EF_STREAMS=1 timeout -k 10 240 python -u $B > $O/rag_new_s1.log 2>&1
ACOSS_EF_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rag_kt -o run -- python3 -u $B --max-pairs 2000000 > $O/rag_kt.log 2>&1
ACOSS_EF_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ef446_kt -o run -- python3 -u tools/ef_bench.py --reps 2 > $O/ef446_kt.log 2>&1
