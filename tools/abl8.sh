set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in base HEAD; do
  if [ $v = base ]; then L=acoss-1_amd/acoss/lib/libacoss_hip.so; else L=tools/abl/libabl_$v.so; fi
  echo "variant=$v"; ACOSS_FUSE_ROWS=0 ACOSS_SPLIT_STREAMS=1 ACOSS_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"
  ACOSS_FUSE_ROWS=0 ACOSS_SPLIT_STREAMS=1 ACOSS_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/abl8/$v -o run -- python3 tools/kbench.py --pairs 2000 --reps 1 > gpurun_out/abl8_$v.log 2>&1
done
