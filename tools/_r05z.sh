set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
ROUNDS=3 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_rowsnt.so" -- --workload c1 > gpurun_out/ab_c1_r05z.txt 2>&1
echo "== c1"; cat gpurun_out/ab_c1_r05z.txt
ROUNDS=3 timeout -k 10 700 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_st0.so" > gpurun_out/ab_c3_r05z.txt 2>&1
echo "== c3"; cat gpurun_out/ab_c3_r05z.txt
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_st0.so" -- --workload c4 > gpurun_out/ab_c4_r05z.txt 2>&1
echo "== c4"; cat gpurun_out/ab_c4_r05z.txt
for v in "CC_X=0" "CC_LIB_PATH=tools/ab/lib_ntload0.so" "CC_X=0" "CC_LIB_PATH=tools/ab/lib_ntload0.so"; do env $v timeout -k 10 200 python -u tools/bench_threshold.py > gpurun_out/thr_r05z.json 2> gpurun_out/thr_r05z.err; echo "thr [$v] $(python3 -c "import json; d=json.loads(open('gpurun_out/thr_r05z.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('kernels_ms', d.get('kernels_ms_per_step')))" | cut -c1-200)"; done
