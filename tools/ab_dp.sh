set -euo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_crp.py tests/test_gpu_plugin.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dp_tests.log 2>&1 || { tail -30 gpurun_out/dp_tests.log; exit 1; }
tail -1 gpurun_out/dp_tests.log
for V in 0 1 0; do
  if [ $V = 1 ]; then export ACOSS_DP_NOFAST=1; else unset ACOSS_DP_NOFAST || true; fi
  echo "ACOSS_DP_NOFAST=$V"
  timeout -k 10 120 python tools/kbench.py --frames 2000 --pairs 13366 --reps 3 2>&1 | grep -E "rep 2|checksum"
done
unset ACOSS_DP_NOFAST
echo "frames=500"; timeout -k 10 120 python tools/kbench.py --frames 500 --pairs 13366 --reps 3 2>&1 | grep -E "rep 2|checksum"
