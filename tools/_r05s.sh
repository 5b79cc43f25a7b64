set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
tools/gpu_steps.sh r05s tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05s.log 2>&1; tail -4 gpurun_out/smoke_r05s.log
tools/gpu_steps.sh r05s bench_full bench_c4 bench_c2 bench_c1 bench_cont
