set -e
cd $GRAFT_REPO_ROOT
for WS in 2147483648 8589934592 17179869184; do echo "ws=$WS"; ACOSS_WS_BYTES=$WS timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"; done
