set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_parity.py tests/test_threshold.py tests/test_gpu_sharded.py > gpurun_out/t_r05u.log 2>&1 || { tail -40 gpurun_out/t_r05u.log; exit 1; }
tail -2 gpurun_out/t_r05u.log
ROUNDS=3 timeout -k 10 700 tools/gpu_ab.sh "CC_X=0" "CC_SAMPLE_ROWS=0" "CC_LIB_PATH=tools/ab/lib_e86b702.so" > gpurun_out/ab_c3_r05u.txt 2>&1
cat gpurun_out/ab_c3_r05u.txt
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_SAMPLE_ROWS=0" -- --workload c2 > gpurun_out/ab_c2_r05u.txt 2>&1
cat gpurun_out/ab_c2_r05u.txt
for v in 1 0; do CC_SAMPLE_ROWS=$v timeout -k 10 200 python -u tools/bench_threshold.py > gpurun_out/thr_r05u_$v.json 2> gpurun_out/thr_r05u.err; echo "rows=$v $(tail -1 gpurun_out/thr_r05u_$v.json | cut -c1-300)"; done
