set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
ROUNDS=3 timeout -k 10 600 tools/gpu_ab.sh "CC_X=0" "CC_PASS2_ORDER=2" "CC_PASS2_ORDER=1" -- --workload c2 > gpurun_out/ab_c2_r05ak.txt 2>&1
echo "== c2"; cat gpurun_out/ab_c2_r05ak.txt
for v in 0 2 0 2; do CC_PASS2_ORDER=$v timeout -k 10 300 python -u tools/bench_sharded_slabs.py 8 c3 10 > gpurun_out/slabs_r05ak.json 2> gpurun_out/slabs_r05ak.err; echo "order $v $(python3 -c "import json; d=json.loads(open('gpurun_out/slabs_r05ak.json').read().strip().splitlines()[-1]); print(d['per_slab_ms'], d['ratio_to_ideal'], d['single_volume_step_ms'])")"; done
