set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_crp.py -x -q -m gpu 2>&1 | tail -1
for v in base PB; do
  if [ $v = base ]; then L=acoss-1_amd/acoss/lib/libacoss_hip.so; else L=tools/abl/libabl_$v.so; fi
  for C in 1 2 4; do
    echo "variant=$v cpw=$C"; ACOSS_COLS_PER_WAVE=$C ACOSS_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"
  done
done
