set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
tools/gpu_steps.sh r05t prof_c3 prof_c4 prof_cont prof_c2 prof_c1 slabs8_c3 slabs8_c4 n2gloo n4gloo
