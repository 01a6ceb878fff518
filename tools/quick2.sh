set -e
cd $GRAFT_REPO_ROOT
for KB in 536870912 2147483648 4294967296; do echo "keybytes=$KB"; ACOSS_KEY_BYTES=$KB timeout -k 10 120 python tools/kbench.py --pairs 6000 --reps 2 2>&1 | grep -E "rep 1"; done
