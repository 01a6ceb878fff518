set -e
export TMPDIR=/tmp
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_earlyfusion_pin.py > $O/pin.log 2>&1
B="tools/bench_datacos.py --algo earlyfusion --frames 47 --blocks-lo 14 --max-pairs 8000000"
timeout -k 10 240 python -u $B > $O/s_warm.log 2>&1
for v in colpack new colpack new; do if [ $v = colpack ]; then L=tools/abl/libabl_colpack.so; else L=acoss-1_amd/acoss/lib/libacoss_hip.so; fi; ACOSS_HIP_LIB=$L timeout -k 10 240 python -u $B > $O/s_$v.$RANDOM.log 2>&1; done
B="tools/bench_datacos.py --algo earlyfusion --frames 80 --blocks-lo 30 --max-pairs 4000000"
for v in colpack new colpack new; do if [ $v = colpack ]; then L=tools/abl/libabl_colpack.so; else L=acoss-1_amd/acoss/lib/libacoss_hip.so; fi; ACOSS_HIP_LIB=$L timeout -k 10 240 python -u $B > $O/m_$v.$RANDOM.log 2>&1; done
ACOSS_EF_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 -u tools/bench_datacos.py --algo earlyfusion --frames 47 --blocks-lo 14 --max-pairs 1000000 > $O/kt.log 2>&1
