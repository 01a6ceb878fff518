set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_simple
mkdir -p $O
cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/tools/simple_one.py 2000 40 1 > $O/kt.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $O/sq -o run -- python3 $R/tools/simple_one.py 2000 40 1 > $O/sq.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM --output-format csv -d $O/sq2 -o run -- python3 $R/tools/simple_one.py 2000 40 1 > $O/sq2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d $O/ta -o run -- python3 $R/tools/simple_one.py 2000 40 1 > $O/ta.log 2>&1 || true
echo done
