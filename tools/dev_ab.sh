#!/bin/bash
# dev A/B timing: current library vs variant libraries (CC_LIB_PATH), interleaved on one box
mkdir -p gpurun_out
B="timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $BENCH_ARGS"
for r in 1 2; do
  $B > gpurun_out/ab_cur_$r.json || exit 1
  for v in scratch/var/*.so; do
    n=$(basename $v .so)
    CC_LIB_PATH=$v $B > gpurun_out/ab_${n}_$r.json || exit 1
  done
done
