set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
ROUNDS=3 timeout -k 10 700 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_dz16.so" "CC_LIB_PATH=tools/ab/lib_dz8.so" > gpurun_out/ab_c3_r05v.txt 2>&1
cat gpurun_out/ab_c3_r05v.txt
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_dz16.so" "CC_LIB_PATH=tools/ab/lib_dz8.so" -- --dither > gpurun_out/ab_cont_r05v.txt 2>&1
cat gpurun_out/ab_cont_r05v.txt
python3 - <<'PY'
import json
for j in range(3):
    d = json.loads(open('gpurun_out/ab_%d.json' % j).read().strip().splitlines()[-1])
    print(j, 'relabelled tiles', d['result'].get('n_relabelled_tiles'), 'k_fix', d['kernels_ms_per_step'].get('k_fix'))
PY
