# k_seams variant: parity (parity + sharded files), same-box A/B against the committed build, PMC
set -e -o pipefail
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=${1:-seamsv2}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sharded.py -m gpu -k "not c5 and not c4_scale" > gpurun_out/par_$V.log 2>&1 || { tail -30 gpurun_out/par_$V.log; exit 1; }
tail -1 gpurun_out/par_$V.log
ROUNDS=3 timeout -k 10 600 tools/gpu_ab_libs.sh 346e055 $V > gpurun_out/ab_$V.txt 2>&1; cat gpurun_out/ab_$V.txt
CC_LIB_PATH=$R/tools/ab/lib_$V.so tools/pmc_bench.sh pmc_$V
python3 tools/pmc_table.py gpurun_out/pmc_$V | grep -E "kernel|seams"
