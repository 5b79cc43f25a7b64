set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
ROUNDS=3 timeout -k 10 700 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_HEAD.so" -- --workload c4 > gpurun_out/ab_c4_r05ai.txt 2>&1
echo "== c4"; cat gpurun_out/ab_c4_r05ai.txt
