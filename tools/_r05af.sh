set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_parity.py tests/test_gpu_sharded.py -k "mask or c4 or order or empty" > gpurun_out/t_r05af.log 2>&1 || { tail -40 gpurun_out/t_r05af.log; exit 1; }
tail -2 gpurun_out/t_r05af.log
ROUNDS=3 timeout -k 10 700 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_HEAD.so" -- --workload c4 > gpurun_out/ab_c4_r05af.txt 2>&1
echo "== c4"; cat gpurun_out/ab_c4_r05af.txt
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_HEAD.so" > gpurun_out/ab_c3_r05af.txt 2>&1
echo "== c3"; cat gpurun_out/ab_c3_r05af.txt
