set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_parity.py tests/test_gpu_sharded.py > gpurun_out/t_r05r.log 2>&1 || { tail -40 gpurun_out/t_r05r.log; exit 1; }
tail -2 gpurun_out/t_r05r.log
ROUNDS=3 timeout -k 10 700 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_ced3150.so" "CC_LIB_PATH=tools/ab/lib_stagger.so" > gpurun_out/ab_c3_r05r.txt 2>&1
cat gpurun_out/ab_c3_r05r.txt
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_ced3150.so" -- --workload c2 > gpurun_out/ab_c2_r05r.txt 2>&1
cat gpurun_out/ab_c2_r05r.txt
