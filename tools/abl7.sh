# VALU instructions per kernel for ablated libraries (unfused rows, one stream)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in base NL NG NT; do
  if [ $v = base ]; then L=acoss-1_amd/acoss/lib/libacoss_hip.so; else L=tools/abl/libabl_$v.so; fi
  ACOSS_FUSE_ROWS=0 ACOSS_SPLIT_STREAMS=1 ACOSS_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d gpurun_out/abl7/$v -o run -- python3 tools/kbench.py --pairs 2000 --reps 1 > gpurun_out/abl7_$v.log 2>&1
  echo "variant $v done"
done
