set -e -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_comm.py -k "mask or empty_tiles or c4" > gpurun_out/t_r05k.log 2>&1 || { tail -40 gpurun_out/t_r05k.log; exit 1; }
tail -2 gpurun_out/t_r05k.log
ROUNDS=3 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_7f5d499.so" -- --workload c4 > gpurun_out/ab_c4_r05k.txt 2>&1
cat gpurun_out/ab_c4_r05k.txt
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_7f5d499.so" > gpurun_out/ab_c3_r05k.txt 2>&1
cat gpurun_out/ab_c3_r05k.txt
