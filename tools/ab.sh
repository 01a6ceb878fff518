# A/B of two library builds on the same box: bash tools/ab.sh <libA> <libB> [env...]
set -e
cd $GRAFT_REPO_ROOT
A=$1; B=$2
for i in 1 2; do
  for L in $A $B; do
    echo "lib=$L"; ACOSS_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"
  done
done
