set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
ROUNDS=3 timeout -k 10 900 tools/gpu_ab.sh "CC_X=0" "CC_PASS2_ORDER=1" "CC_PASS2_ORDER=2" "CC_LIB_PATH=tools/ab/lib_mstage0.so" -- --workload c4 > gpurun_out/ab_c4_r05ad.txt 2>&1
cat gpurun_out/ab_c4_r05ad.txt
