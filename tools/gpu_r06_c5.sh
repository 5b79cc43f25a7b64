# C5 slab: k_pass2 tile orders (CC_PASS2_ORDER 0-5), same box, plus C3 for reference
set -e -o pipefail
mkdir -p gpurun_out
ROUNDS=2 timeout -k 10 900 tools/gpu_ab.sh "CC_PASS2_ORDER=0" "CC_PASS2_ORDER=1" "CC_PASS2_ORDER=2" "CC_PASS2_ORDER=3" "CC_PASS2_ORDER=4" "CC_PASS2_ORDER=5" -- --workload c5 > gpurun_out/ab_c5_order6.txt 2>&1; cat gpurun_out/ab_c5_order6.txt
ROUNDS=1 timeout -k 10 300 tools/gpu_ab.sh "CC_PASS2_ORDER=0" "CC_PASS2_ORDER=3" -- --workload c3 > gpurun_out/ab_c3_order.txt 2>&1; cat gpurun_out/ab_c3_order.txt
