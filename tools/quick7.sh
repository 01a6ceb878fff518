set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_gpu_crp.py -x -q -m gpu 2>&1 | tail -2
timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2|checksum"
ACOSS_SPLIT_STREAMS=1 timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 3 2>&1 | grep -E "rep 2"
