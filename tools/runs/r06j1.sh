set -e
export TMPDIR=/tmp
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 900 bash profiles/profile.sh r06j > $O/profile.log 2>&1
timeout -k 10 400 python -u tools/datacos_plugin.py --algo simple --tracks 15000 --out $O/datacos_simple_15000.json > $O/datacos_simple_15000.txt 2>&1
