# Same-box A/B of launch folds (tools/ab/lib_BASE.so vs lib_VARIANT.so): the tree's library (the
# variant) through the parity, sharded, comm and mask files first, then round-robin 8-slab C3
# schedule lines and C2 / C3 bench lines.  Usage: tools/gpu_r06_fold.sh BASE VARIANT
set -e -o pipefail
mkdir -p gpurun_out
B=$1; V=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_comm.py tests/test_gpu_comm_ranks.py tests/test_gpu_mask_live.py -m gpu -k "not c4_scale" > gpurun_out/fold_tests_$V.log 2>&1 || { tail -30 gpurun_out/fold_tests_$V.log; exit 1; }
tail -1 gpurun_out/fold_tests_$V.log
for i in 1 2 3; do
  for n in $B $V; do
    CC_LIB_PATH=$ROOT/tools/ab/lib_$n.so timeout -k 10 200 python -u tools/bench_sharded_slabs.py 8 c3 10 > gpurun_out/fold_slabs_$n.json 2> gpurun_out/fold_slabs_$n.err
    python3 -c "
import json; d=json.loads(open('gpurun_out/fold_slabs_$n.json').read().strip().splitlines()[-1])
k=d['middle_slab_kernels_ms']; print('$n slabs8', d['per_slab_ms'], d['ratio_to_ideal'], len(k), round(sum(k.values()),4))"
  done
done
ROUNDS=3 timeout -k 10 400 tools/gpu_ab_libs.sh $B $V -- --workload c2 --steps 50 --warmup 10
ROUNDS=2 timeout -k 10 400 tools/gpu_ab_libs.sh $B $V -- --workload c3
