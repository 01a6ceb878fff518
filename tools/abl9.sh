set -e
cd $GRAFT_REPO_ROOT
for v in base O3; do
  if [ $v = base ]; then L=acoss-1_amd/acoss/lib/libacoss_hip.so; else L=tools/abl/libabl_$v.so; fi
  for S in 1 2; do echo "variant=$v streams=$S"; ACOSS_SPLIT_STREAMS=$S ACOSS_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"; done
done
