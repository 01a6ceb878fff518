set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_crp.py -x -q -m gpu 2>&1 | tail -2
for C in 1 2 4 8; do echo "cpw=$C"; ACOSS_COLS_PER_WAVE=$C timeout -k 10 120 python tools/kbench.py --frames 2000 --pairs 13366 --reps 3 2>&1 | grep -E "rep 2|checksum"; done
echo "frames=500 cpw=4"; ACOSS_COLS_PER_WAVE=4 timeout -k 10 120 python tools/kbench.py --frames 500 --pairs 13366 --reps 3 2>&1 | grep -E "rep 2|checksum"
