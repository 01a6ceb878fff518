set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_crp.py -x -q -m gpu 2>&1 | tail -3
for P in split fused; do echo "path=$P"; ACOSS_CRP_PATH=$P timeout -k 10 120 python tools/kbench.py --pairs 4000 --reps 2 2>&1 | grep -E "rep 1|checksum"; done
