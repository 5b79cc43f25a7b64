set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
tools/gpu_steps.sh r05ao bench_full bench_c4 bench_c2 bench_c1
