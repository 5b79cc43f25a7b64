set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
ROUNDS=3 timeout -k 10 700 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_ntload.so" > gpurun_out/ab_c3_r05w.txt 2>&1
cat gpurun_out/ab_c3_r05w.txt
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_ntload.so" -- --workload c4 > gpurun_out/ab_c4_r05w.txt 2>&1
cat gpurun_out/ab_c4_r05w.txt
