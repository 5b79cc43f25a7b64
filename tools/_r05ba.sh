set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
ROUNDS=3 bash tools/gpu_ab_libs.sh base h7 h9 -- --warmup 3 > gpurun_out/ab_r05ba.txt 2>&1
cat gpurun_out/ab_r05ba.txt
