#!/bin/bash
# dev loop: GPU parity tests, two C3 bench runs, the ablation harness (each step time-limited)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
B="timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
$B > gpurun_out/q1.json || exit 1
$B > gpurun_out/q2.json || exit 1
$B --mode less > gpurun_out/q3.json || exit 1
timeout -k 10 120 tools/ablate 1024 2048 2048 64 512 512 0 10 > gpurun_out/ablate.txt 2>&1 || exit 1
