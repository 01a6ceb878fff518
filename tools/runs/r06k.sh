set -e
export TMPDIR=/tmp
O=gpurun_out/r06k; mkdir -p $O
ACOSS_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 > $O/bench_gloo2.json 2> $O/bench_gloo2.err
