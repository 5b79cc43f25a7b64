set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_parity.py tests/test_threshold.py tests/test_gpu_comm.py > gpurun_out/t_r05y.log 2>&1 || { tail -40 gpurun_out/t_r05y.log; exit 1; }
tail -2 gpurun_out/t_r05y.log
ROUNDS=3 timeout -k 10 700 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_ntload0.so" > gpurun_out/ab_c3_r05y.txt 2>&1
cat gpurun_out/ab_c3_r05y.txt
for w in c2 c1 c4; do ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_ntload0.so" -- --workload $w > gpurun_out/ab_${w}_r05y.txt 2>&1; echo "== $w"; cat gpurun_out/ab_${w}_r05y.txt; done
for v in "CC_X=0" "CC_LIB_PATH=tools/ab/lib_ntload0.so" "CC_X=0" "CC_LIB_PATH=tools/ab/lib_ntload0.so"; do env $v timeout -k 10 200 python -u tools/bench_threshold.py > gpurun_out/thr_r05y.json 2> gpurun_out/thr_r05y.err; echo "thr [$v] $(tail -1 gpurun_out/thr_r05y.json | cut -c1-260)"; done
