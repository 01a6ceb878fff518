set -e
cd $GRAFT_REPO_ROOT
for KB in 268435456 536870912 1073741824 2147483648; do echo "key_bytes=$KB"; ACOSS_KEY_BYTES=$KB timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"; done
