set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_threshold.py > gpurun_out/t_r05x.log 2>&1 || { tail -40 gpurun_out/t_r05x.log; exit 1; }
tail -2 gpurun_out/t_r05x.log
ROUNDS=3 timeout -k 10 800 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_rdnt.so" "CC_LIB_PATH=tools/ab/lib_rdnt_st.so" "CC_LIB_PATH=tools/ab/lib_ntload0.so" > gpurun_out/ab_c3_r05x.txt 2>&1
cat gpurun_out/ab_c3_r05x.txt
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_SPEC_STAGGER=0" "CC_LIB_PATH=tools/ab/lib_rdnt.so" -- --workload c2 > gpurun_out/ab_c2_r05x.txt 2>&1
cat gpurun_out/ab_c2_r05x.txt
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_rdnt.so" -- --workload c4 > gpurun_out/ab_c4_r05x.txt 2>&1
cat gpurun_out/ab_c4_r05x.txt
for v in 1 0 1 0; do CC_SPEC_STAGGER=$v timeout -k 10 300 python -u tools/bench_sharded_slabs.py 8 c3 10 > gpurun_out/slabs_r05x.json 2> gpurun_out/slabs_r05x.err; echo "stagger $v $(python3 -c "import json; d=json.loads(open('gpurun_out/slabs_r05x.json').read().strip().splitlines()[-1]); print(d['per_slab_ms'], d['ratio_to_ideal'], d['single_volume_step_ms'])")"; done
