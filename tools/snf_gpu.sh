set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_plugin.py -m gpu -x -v --timeout 120 --timeout-method thread -k snf > gpurun_out/snf_tests.log 2>&1 || { tail -40 gpurun_out/snf_tests.log; exit 1; }
tail -2 gpurun_out/snf_tests.log
timeout -k 10 200 python -u tools/bench_snf.py --n 2000 --L 2 --K 20 > gpurun_out/snf_bench.json
timeout -k 10 200 python -u tools/bench_snf.py --n 15000 --L 2 --K 20 >> gpurun_out/snf_bench.json
timeout -k 10 200 python -u tools/bench_snf.py --n 15000 --L 4 --K 20 >> gpurun_out/snf_bench.json
cat gpurun_out/snf_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_snf -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_snf.py --n 15000 --L 2 --K 20 --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_snf.log 2>&1
echo profiled
