set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_crp.py -x -q -m gpu 2>&1 | tail -3
for A in 0 2; do echo "ablate=$A"; ACOSS_DEBUG_ABLATE=$A timeout -k 10 120 python tools/kbench.py --pairs 4000 --reps 2 2>&1 | grep -E "rep|checksum"; done
