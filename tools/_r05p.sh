set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_SPEC_STAGGER_US=0" "CC_SPEC_STAGGER_US=6" "CC_SPEC_STAGGER_US=12" "CC_SPEC_STAGGER_US=20" -- --workload c2 > gpurun_out/ab_c2_r05p.txt 2>&1
cat gpurun_out/ab_c2_r05p.txt
ROUNDS=2 timeout -k 10 600 tools/gpu_ab.sh "CC_SPEC_STAGGER_US=0" "CC_SPEC_STAGGER_US=6" "CC_SPEC_STAGGER_US=12" -- --workload c1 > gpurun_out/ab_c1_r05p.txt 2>&1
cat gpurun_out/ab_c1_r05p.txt
for v in 0 12 0 12; do CC_SPEC_STAGGER_US=$v timeout -k 10 300 python -u tools/bench_sharded_slabs.py 8 c3 10 > gpurun_out/slabs_r05p_$v.json 2> gpurun_out/slabs_r05p.err; echo "stagger $v $(tail -1 gpurun_out/slabs_r05p_$v.json)"; done
