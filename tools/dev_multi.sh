mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 150 --timeout-method thread > gpurun_out/sharded.log 2>&1 || { tail -40 gpurun_out/sharded.log; exit 1; }
tail -3 gpurun_out/sharded.log
CC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --shape 256,2048,2048 --steps 5 --warmup 2 > gpurun_out/bench_rehearsal2.json 2> gpurun_out/bench_rehearsal2.err || { tail -30 gpurun_out/bench_rehearsal2.err; exit 1; }
cat gpurun_out/bench_rehearsal2.json
