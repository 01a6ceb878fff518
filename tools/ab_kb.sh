set -euo pipefail
cd "$GRAFT_REPO_ROOT"
for KB in 536870912 805306368 1073741824 1610612736 2147483648; do
  echo "ACOSS_KEY_BYTES=$KB"
  ACOSS_KEY_BYTES=$KB timeout -k 10 120 python tools/kbench.py --frames 2000 --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"
done
