set -e
export TMPDIR=/tmp
O=gpurun_out/r06z; mkdir -p $O
B="tools/bench_datacos.py --algo earlyfusion --frames 47 --blocks-lo 14 --max-pairs 12000000"
timeout -k 10 240 python -u $B > $O/rag_warm.log 2>&1
for i in 1 2; do
ACOSS_EF_PACK=0 timeout -k 10 240 python -u $B > $O/rag_nopack$i.log 2>&1
timeout -k 10 240 python -u $B > $O/rag_pack$i.log 2>&1
done
ACOSS_EF_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rag_kt -o run -- python3 -u tools/bench_datacos.py --algo earlyfusion --frames 47 --blocks-lo 14 --max-pairs 2000000 > $O/rag_kt.log 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_earlyfusion_pin.py -k "short" > $O/pin.log 2>&1
