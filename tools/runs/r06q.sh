set -e
export TMPDIR=/tmp
O=gpurun_out/r06q2; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_earlyfusion_pin.py > $O/pin.log 2>&1
B="tools/bench_datacos.py --algo earlyfusion --frames 47 --blocks-lo 14 --max-pairs 8000000"
timeout -k 10 240 python -u $B > $O/s_warm.log 2>&1
for v in 1 2 1 2; do ACOSS_EF_PACK=$v timeout -k 10 240 python -u $B > $O/s_pack$v.$RANDOM.log 2>&1; done
B="tools/bench_datacos.py --algo earlyfusion --frames 80 --blocks-lo 30 --max-pairs 4000000"
for v in 0 2 1 0 2 1; do ACOSS_EF_PACK=$v timeout -k 10 240 python -u $B > $O/m_pack$v.$RANDOM.log 2>&1; done
