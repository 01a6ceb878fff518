set -e
export TMPDIR=/tmp
O=gpurun_out/r06x2; mkdir -p $O
for b in 4096 2048 1024 512 256 128; do ACOSS_EF_BYTES=$((b<<20)) timeout -k 10 120 python -u tools/ef_bench.py --reps 4 > $O/ef_$b.log 2>&1; done
for b in 1024 256; do ACOSS_EF_STREAMS=1 ACOSS_EF_BYTES=$((b<<20)) timeout -k 10 120 python -u tools/ef_bench.py --reps 4 > $O/ef1s_$b.log 2>&1; done
