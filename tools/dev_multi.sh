#!/bin/bash
# dev: GPU tests (all), then the N = 2 bench schedule rehearsed with two ranks on one GPU (gloo)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
CC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --shape 256,2048,2048 --steps 5 --warmup 2 > gpurun_out/bench_rehearsal2.json 2> gpurun_out/bench_rehearsal2.err || { tail -30 gpurun_out/bench_rehearsal2.err; exit 1; }
cut -c 1-300 gpurun_out/bench_rehearsal2.json
