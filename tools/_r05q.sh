set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_SPEC_STAGGER_US=4" "CC_SPEC_STAGGER_US=6" "CC_SPEC_STAGGER_US=9" "CC_SPEC_STAGGER_US=6 CC_PASS2_STAGGER_US=4" "CC_SPEC_STAGGER_US=6 CC_PASS2_STAGGER_US=8" -- --workload c2 > gpurun_out/ab_c2_r05q.txt 2>&1
cat gpurun_out/ab_c2_r05q.txt
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_ced3150.so" > gpurun_out/ab_c3_r05q.txt 2>&1
cat gpurun_out/ab_c3_r05q.txt
for v in "0 0" "6 0" "6 6" "0 0" "6 0" "6 6"; do set -- $v; CC_SPEC_STAGGER_US=$1 CC_PASS2_STAGGER_US=$2 timeout -k 10 300 python -u tools/bench_sharded_slabs.py 8 c3 10 > gpurun_out/slabs_r05q.json 2> gpurun_out/slabs_r05q.err; echo "stagger $1 $2 $(python3 -c "import json; d=json.loads(open('gpurun_out/slabs_r05q.json').read().strip().splitlines()[-1]); print(d['per_slab_ms'], d['ratio_to_ideal'], d['single_volume_step_ms'])")"; done
