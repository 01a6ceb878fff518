set -e
cd $GRAFT_REPO_ROOT
for v in base NR2 NG; do
  if [ $v = base ]; then L=acoss-1_amd/acoss/lib/libacoss_hip.so; else L=tools/abl/libabl_$v.so; fi
  echo "variant=$v"; ACOSS_SPLIT_STREAMS=1 ACOSS_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"
done
