set -e -o pipefail
mkdir -p gpurun_out
tools/gpu_steps.sh r05m tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05m.log 2>&1; tail -5 gpurun_out/smoke_r05m.log
ROUNDS=3 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_nt0.so" > gpurun_out/ab_c3_r05m.txt 2>&1
cat gpurun_out/ab_c3_r05m.txt
