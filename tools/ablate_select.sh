set -e
cd $GRAFT_REPO_ROOT
for A in 0 1 2 3; do echo "ablate=$A"; ACOSS_DEBUG_ABLATE=$A timeout -k 10 120 python tools/kbench.py --pairs 4000 --reps 2 2>&1 | grep rep; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_sel -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --pairs 4000 --reps 1 > gpurun_out/prof_sel.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_sel2 -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --pairs 4000 --reps 1 > gpurun_out/prof_sel2.log 2>&1
