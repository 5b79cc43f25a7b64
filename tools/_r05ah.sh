set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
tools/gpu_steps.sh r05ah roof bench_full bench_c4 bench_c2 bench_c1 bench_cont slabs8_c3 slabs8_c4 n2gloo
