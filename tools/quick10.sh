set -e
cd $GRAFT_REPO_ROOT
for F in 500 50; do echo "frames=$F"; timeout -k 10 120 python tools/kbench.py --frames $F --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"; done
echo "frames=2000 dmax"; timeout -k 10 120 python tools/kbench.py --frames 2000 --pairs 13366 --reps 3 --dmax 2>&1 | grep -E "rep 2"
