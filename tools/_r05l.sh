set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/graph_probe 300 14 > gpurun_out/graph_probe_r05l.txt 2>&1; cat gpurun_out/graph_probe_r05l.txt
timeout -k 10 120 tools/graph_probe 300 4 >> gpurun_out/graph_probe_r05l.txt 2>&1; tail -6 gpurun_out/graph_probe_r05l.txt
ROUNDS=3 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_nt.so" > gpurun_out/ab_c3_r05l.txt 2>&1
cat gpurun_out/ab_c3_r05l.txt
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_nt.so" -- --workload c4 > gpurun_out/ab_c4_r05l.txt 2>&1
cat gpurun_out/ab_c4_r05l.txt
