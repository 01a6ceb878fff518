set -e
cd $GRAFT_REPO_ROOT
for cfg in "2 1073741824" "1 1073741824" "2 536870912" "2 2147483648" "1 2147483648"; do
  set -- $cfg
  echo "streams=$1 key=$2"; ACOSS_SPLIT_STREAMS=$1 ACOSS_KEY_BYTES=$2 timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"
done
