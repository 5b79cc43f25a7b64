set -e -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_comm.py -k "front_variants or speculated or continuous or fused_path_golden or c3_vs_oracle or both_schedules or single_gpu_vs_oracle or root_capacity or comm or c1_shape or white_noise" > gpurun_out/t_r05f.log 2>&1 || { tail -40 gpurun_out/t_r05f.log; exit 1; }
tail -2 gpurun_out/t_r05f.log
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/sd_r05f.json 2>/dev/null
KS=$(python3 -c "import json; d = json.loads(open('gpurun_out/sd_r05f.json').read().strip().splitlines()[-1]); print(d['kernels_ms_per_step']['k_spec'])")
echo "k_spec $KS"
if python3 -c "import sys; sys.exit(0 if $KS > 3.45 else 1)"; then
  echo SLOW
  ROUNDS=2 timeout -k 10 800 tools/gpu_ab.sh "CC_LIB_PATH=tools/ab/lib_b436cb4.so" "CC_LIB_PATH=tools/ab/lib_b5c4e22.so CC_SPEC_TILESTATS=0 CC_SPEC_TBFREE=0" "CC_SPEC_TILESTATS=0 CC_SPEC_TBFREE=0" "CC_SPEC_TILESTATS=1 CC_SPEC_TBFREE=0" "CC_SPEC_TILESTATS=0 CC_SPEC_TBFREE=1" "CC_SPEC_TILESTATS=1 CC_SPEC_TBFREE=1" > gpurun_out/ab_slow_r05f.txt 2>&1 || true
  cat gpurun_out/ab_slow_r05f.txt
  tools/gpu_steps.sh r05f slowdiag
else
  echo FAST
  ROUNDS=3 timeout -k 10 600 tools/gpu_ab.sh "CC_LIB_PATH=tools/ab/lib_b5c4e22.so CC_SPEC_TILESTATS=0 CC_SPEC_TBFREE=0" "CC_SPEC_TILESTATS=0 CC_SPEC_TBFREE=0" "CC_SPEC_TILESTATS=1 CC_SPEC_TBFREE=1" -- --workload c2 --steps 30 > gpurun_out/ab_fast_r05f.txt 2>&1 || true
  cat gpurun_out/ab_fast_r05f.txt
fi
