#!/bin/bash
# dev A/B timing: current library vs scratch/old (built from an earlier commit), same box
mkdir -p gpurun_out
B="timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
$B > gpurun_out/ab_new2.json || exit 1
$B --timed-prof 1 > gpurun_out/ab_new1.json || exit 1
CC_LIB_PATH=scratch/old/libcc_mi355x.so $B > gpurun_out/ab_old.json || exit 1
$B > gpurun_out/ab_new2b.json || exit 1
CC_LIB_PATH=scratch/old/libcc_mi355x.so $B > gpurun_out/ab_oldb.json || exit 1
