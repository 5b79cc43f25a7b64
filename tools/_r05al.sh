set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
tools/gpu_steps.sh r05al trace_slabs8
python3 tools/trace_gaps.py gpurun_out/trace_slabs8_r05al > gpurun_out/trace_slabs8_r05al_summary.txt 2>&1 || true
head -40 gpurun_out/trace_slabs8_r05al_summary.txt
