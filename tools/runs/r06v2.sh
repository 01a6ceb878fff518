set -e
export TMPDIR=/tmp
O=gpurun_out/r06v2; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_earlyfusion_pin.py > $O/pin.log 2>&1
timeout -k 10 120 python -u tools/ef_bench.py --reps 3 > $O/ef.log 2>&1
ACOSS_EF_STREAMS=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 -u tools/ef_bench.py --reps 1 > $O/kt.log 2>&1
