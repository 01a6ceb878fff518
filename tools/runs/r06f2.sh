set -e
export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 400 python -u tools/datacos_plugin.py --algo simple --tracks 15000 --out $O/datacos_simple_15000.json > $O/datacos_simple_15000.txt 2>&1
timeout -k 10 400 python -u tools/datacos_plugin.py --algo serra09 --tracks 15000 --out $O/datacos_serra09_15000.json > $O/datacos_serra09_15000.txt 2>&1
