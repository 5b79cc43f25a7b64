set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
tools/gpu_steps.sh r05ag tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05ag.log 2>&1; tail -4 gpurun_out/smoke_r05ag.log
tools/gpu_steps.sh r05ag prof_c3 prof_c4 prof_cont prof_c2 prof_c1
