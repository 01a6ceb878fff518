set -e
export TMPDIR=/tmp
O=gpurun_out/r06z6; mkdir -p $O
timeout -k 10 120 python -u tools/ef_bench.py --reps 4 > $O/ef.log 2>&1
ACOSS_EF_STREAMS=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 -u tools/ef_bench.py --reps 1 > $O/kt.log 2>&1
ACOSS_EF_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kts -o run -- python3 -u tools/bench_datacos.py --algo earlyfusion --frames 47 --blocks-lo 14 --max-pairs 1000000 > $O/kts.log 2>&1
