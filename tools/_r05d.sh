set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "front_variants or speculated or sign_bit or continuous_synthetic or synthetic_vs_oracle or mask_vs_oracle or fused_path_golden or c3_vs_oracle or c3_continuous or c3_mask or both_schedules" > gpurun_out/t_r05d.log 2>&1 || { tail -30 gpurun_out/t_r05d.log; exit 1; }
tail -2 gpurun_out/t_r05d.log
ROUNDS=3 timeout -k 10 600 tools/gpu_ab.sh "CC_LIB_PATH=tools/ab/lib_b436cb4.so" "CC_SPEC_TILESTATS=0 CC_SPEC_TBFREE=0" "CC_SPEC_TILESTATS=1 CC_SPEC_TBFREE=0" "CC_SPEC_TILESTATS=0 CC_SPEC_TBFREE=1" "CC_SPEC_TILESTATS=1 CC_SPEC_TBFREE=1" > gpurun_out/ab_r05d.txt 2>&1
cat gpurun_out/ab_r05d.txt
tools/gpu_steps.sh r05d slowdiag
