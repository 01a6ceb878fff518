set -e
export TMPDIR=/tmp
O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_earlyfusion_pin.py > $O/pin.log 2>&1
timeout -k 10 300 python -u tools/datacos_plugin.py --algo earlyfusion --frames 240 --beat-period 5 --tracks 15000 --out $O/datacos_earlyfusion_15000.json > $O/datacos_earlyfusion_15000.txt 2>&1
timeout -k 10 300 python -u tools/datacos_plugin.py --algo earlyfusion --frames 500 --beat-period 7 --tracks 15000 --out $O/datacos_earlyfusion_15000_b7.json > $O/datacos_earlyfusion_15000_b7.txt 2>&1
