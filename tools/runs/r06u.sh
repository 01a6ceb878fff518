set -e
export TMPDIR=/tmp
O=gpurun_out/r06u; mkdir -p $O
B="tools/ef_bench.py --reps 1"
ACOSS_EF_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $O/sq -o run -- python3 -u $B > $O/sq.log 2>&1
ACOSS_EF_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TCP_TCC_READ_REQ_sum --output-format csv -d $O/tcc -o run -- python3 -u $B > $O/tcc.log 2>&1
ACOSS_EF_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM --output-format csv -d $O/sq2 -o run -- python3 -u $B > $O/sq2.log 2>&1
ACOSS_EF_STREAMS=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 -u $B > $O/kt.log 2>&1
