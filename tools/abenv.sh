# A/B of an env switch on the same box: bash tools/abenv.sh VAR valA valB
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_gpu_crp.py -x -q -m gpu 2>&1 | tail -1
for i in 1 2; do
  for v in $2 $3; do
    echo "$1=$v"; env $1=$v timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"
  done
done
