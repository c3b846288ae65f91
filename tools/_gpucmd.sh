export TMPDIR=/tmp
export PKD_BENCH_SHARE_GPU=1 PKD_BENCH_BACKEND=gloo
python tools/gpu_steps.py \
  bench2 300 'python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1' \
  bench4 300 'python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 4 --steps 3 --warmup 1'
