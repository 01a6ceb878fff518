set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_gpu_crp.py tests/test_gpu_plugin.py -x -q -m gpu 2>&1 | tail -3
for KB in 2147483648 536870912 268435456; do echo "key_bytes=$KB"; ACOSS_KEY_BYTES=$KB timeout -k 10 120 python tools/kbench.py --pairs 13366 --reps 2 2>&1 | grep -E "rep 1|checksum"; done
