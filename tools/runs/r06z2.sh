set -e
export TMPDIR=/tmp
O=gpurun_out/r06z2; mkdir -p $O
B="tools/bench_datacos.py --algo earlyfusion --frames 47 --blocks-lo 14 --max-pairs 500000"
for v in 0 1; do
ACOSS_EF_PACK=$v ACOSS_EF_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA --output-format csv -d $O/sq$v -o run -- python3 -u $B > $O/sq$v.log 2>&1
ACOSS_EF_PACK=$v ACOSS_EF_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TA_BUSY_avr --output-format csv -d $O/f$v -o run -- python3 -u $B > $O/f$v.log 2>&1
done
