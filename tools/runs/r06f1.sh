set -e
export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 900 bash profiles/profile.sh r06f > $O/profile.log 2>&1
timeout -k 10 300 python -u tools/datacos_plugin.py --algo earlyfusion --frames 240 --beat-period 5 --tracks 15000 --out $O/datacos_earlyfusion_15000.json > $O/datacos_earlyfusion_15000.txt 2>&1
timeout -k 10 300 python -u tools/datacos_plugin.py --algo earlyfusion --frames 500 --beat-period 7 --tracks 15000 --host-eval-keys , --out $O/datacos_earlyfusion_15000_b7.json > $O/datacos_earlyfusion_15000_b7.txt 2>&1
