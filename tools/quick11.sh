set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_crp.py -x -q -m gpu 2>&1 | tail -2
for F in 2000 500; do echo "frames=$F"; timeout -k 10 120 python tools/kbench.py --frames $F --pairs 13366 --reps 3 2>&1 | grep -E "rep 2|checksum"; done
