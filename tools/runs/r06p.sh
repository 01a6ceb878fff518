set -e
export TMPDIR=/tmp
O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_earlyfusion_pin.py > $O/pin.log 2>&1
B="tools/bench_datacos.py --algo earlyfusion --frames 47 --blocks-lo 14 --max-pairs 12000000"
timeout -k 10 240 python -u $B > $O/rag_warm.log 2>&1
for i in 1 2; do
ACOSS_EF_PACK=0 timeout -k 10 240 python -u $B > $O/rag_nopack$i.log 2>&1
timeout -k 10 240 python -u $B > $O/rag_pack$i.log 2>&1
done
timeout -k 10 300 python -u tools/datacos_plugin.py --algo earlyfusion --frames 240 --beat-period 5 --tracks 15000 --out $O/datacos_earlyfusion_15000.json > $O/datacos_earlyfusion_15000.txt 2>&1
timeout -k 10 300 python -u tools/datacos_plugin.py --algo earlyfusion --frames 500 --beat-period 7 --tracks 15000 --host-eval-keys , --out $O/datacos_earlyfusion_15000_b7.json > $O/datacos_earlyfusion_15000_b7.txt 2>&1
