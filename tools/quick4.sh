set -e
cd $GRAFT_REPO_ROOT
for KB in 2147483648 4294967296 8589934592; do echo "key_bytes=$KB"; ACOSS_KEY_BYTES=$KB timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 2 2>&1 | grep -E "rep 1|checksum"; done
