set -e
cd $GRAFT_REPO_ROOT
for KB in 402653184 671088640 1073741824 1610612736 2147483648; do
  for F in 2000 500; do echo "kbytes=$KB frames=$F"; ACOSS_KEY_BYTES=$KB timeout -k 10 120 python tools/kbench.py --frames $F --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"; done
done
