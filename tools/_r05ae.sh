set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
ROUNDS=2 timeout -k 10 900 tools/gpu_ab.sh "CC_X=0" "CC_PASS2_ORDER=2" "CC_LIB_PATH=tools/ab/lib_mstage0.so" "CC_LIB_PATH=tools/ab/lib_mstage0.so CC_PASS2_ORDER=2" -- --workload c4 > gpurun_out/ab_c4_r05ae.txt 2>&1
echo "== c4"; cat gpurun_out/ab_c4_r05ae.txt
ROUNDS=3 timeout -k 10 700 tools/gpu_ab.sh "CC_X=0" "CC_PASS2_ORDER=2" > gpurun_out/ab_c3_r05ae.txt 2>&1
echo "== c3"; cat gpurun_out/ab_c3_r05ae.txt
for v in "CC_X=0" "CC_LIB_PATH=tools/ab/lib_auxnt.so" "CC_X=0" "CC_LIB_PATH=tools/ab/lib_auxnt.so"; do
  env $v timeout -k 10 300 python -u tools/bench_prefilter.py --steps 3 > gpurun_out/pf_r05ae.json 2> gpurun_out/pf_r05ae.err; echo "prefilter [$v] $(tail -1 gpurun_out/pf_r05ae.json | cut -c1-400)"
  env $v timeout -k 10 300 python -u tools/bench_misc.py > gpurun_out/misc_r05ae.json 2> gpurun_out/misc_r05ae.err; echo "misc [$v] $(tail -1 gpurun_out/misc_r05ae.json | cut -c1-400)"
  env $v timeout -k 10 300 python -u tools/bench_stage.py > gpurun_out/stage_r05ae.json 2> gpurun_out/stage_r05ae.err; echo "stage [$v] $(tail -1 gpurun_out/stage_r05ae.json | cut -c1-400)"
done
