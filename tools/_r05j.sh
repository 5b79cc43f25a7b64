set -e -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_parity.py tests/test_gpu_sharded.py -k "empty_tiles or mask or speculated or c3_vs_oracle or synthetic_vs_oracle or fused_path_golden or max_runs or white_noise or single_gpu_vs_oracle or unaligned or c1_shape" > gpurun_out/t_r05j.log 2>&1 || { tail -40 gpurun_out/t_r05j.log; exit 1; }
tail -2 gpurun_out/t_r05j.log
ROUNDS=3 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_c1b0725.so" "CC_LIB_PATH=tools/ab/lib_f89f4ef.so" > gpurun_out/ab_c3_r05j.txt 2>&1
cat gpurun_out/ab_c3_r05j.txt
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_f89f4ef.so" -- --workload c4 > gpurun_out/ab_c4_r05j.txt 2>&1
cat gpurun_out/ab_c4_r05j.txt
