set -e -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_comm.py tests/test_gpu_parity.py tests/test_gpu_sharded.py -k "comm or root_capacity or synthetic_vs_oracle or front_variants or c3_vs_oracle or mask_vs_oracle or c3_mask or single_gpu_vs_oracle or without_fast" > gpurun_out/t_r05e.log 2>&1 || { tail -40 gpurun_out/t_r05e.log; exit 1; }
tail -2 gpurun_out/t_r05e.log
CC_LIB_PATH=tools/ab/lib_mstage.so timeout -k 10 300 $T tests/test_gpu_parity.py -k "mask or speculated" > gpurun_out/t_mstage_r05e.log 2>&1 || { tail -40 gpurun_out/t_mstage_r05e.log; exit 1; }
tail -2 gpurun_out/t_mstage_r05e.log
ROUNDS=3 timeout -k 10 400 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_mstage.so" -- --workload c4 > gpurun_out/ab_mstage_r05e.txt 2>&1
cat gpurun_out/ab_mstage_r05e.txt
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/sd_r05e.json 2>/dev/null
KS=$(python3 -c "import json; d = json.loads(open('gpurun_out/sd_r05e.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernels_ms_per_step'])")
echo "bench $KS"
KS=$(python3 -c "import json; d = json.loads(open('gpurun_out/sd_r05e.json').read().strip().splitlines()[-1]); print(d['kernels_ms_per_step']['k_spec'])")
if python3 -c "import sys; sys.exit(0 if $KS > 3.45 else 1)"; then
  echo SLOW
  ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_LIB_PATH=tools/ab/lib_b436cb4.so" "CC_SPEC_TILESTATS=0 CC_SPEC_TBFREE=0" "CC_SPEC_TILESTATS=1 CC_SPEC_TBFREE=0" "CC_SPEC_TILESTATS=0 CC_SPEC_TBFREE=1" "CC_SPEC_TILESTATS=1 CC_SPEC_TBFREE=1" > gpurun_out/ab_slow_r05e.txt 2>&1
  cat gpurun_out/ab_slow_r05e.txt
  tools/gpu_steps.sh r05e slowdiag
else
  echo FAST
fi
