# A/B of library builds on one box, with the Qmax checksum of each (must agree):
#   bash tools/ab2.sh <libA> <libB> ...
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for L in "$@"; do
    echo "lib=$L"; ACOSS_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2|checksum"
  done
done
