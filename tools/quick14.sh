set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_crp.py -x -q -m gpu 2>&1 | tail -1
for C in 1 4 8; do echo "dp_chunks=$C"; ACOSS_DP_CHUNKS=$C timeout -k 10 120 python tools/kbench.py --frames 2000 --pairs 13366 --reps 3 2>&1 | grep -E "rep 2|checksum"; done
echo "frames=500"; timeout -k 10 120 python tools/kbench.py --frames 500 --pairs 13366 --reps 3 2>&1 | grep -E "rep 2|checksum"
echo "frames=2000 dmax"; timeout -k 10 120 python tools/kbench.py --frames 2000 --pairs 13366 --reps 3 --dmax 2>&1 | grep -E "rep 2|checksum"
