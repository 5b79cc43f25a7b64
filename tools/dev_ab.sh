#!/bin/bash
# dev A/B timing: current library vs variant libraries (CC_LIB_PATH), interleaved on one box;
# optional GPU tests first (AB_TESTS=1)
mkdir -p gpurun_out
if [ "${AB_TESTS:-0}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
fi
B="timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $BENCH_ARGS"
for r in 1 2; do
  $B > gpurun_out/ab_cur_$r.json || exit 1
  for v in scratch/var/*.so; do
    n=$(basename $v .so)
    CC_LIB_PATH=$v $B > gpurun_out/ab_${n}_$r.json || exit 1
  done
done
