# Same-box round-robin A/B of the 8-slab C3 schedule (tools/bench_sharded_slabs.py) over library
# builds tools/ab/lib_NAME.so, after the sharded + multi-rank files with the tree's library.
# Usage: tools/gpu_r06_slabs_ab.sh NAME ...   (ROUNDS, default 3)
set -e -o pipefail
mkdir -p gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_comm_ranks.py tests/test_gpu_comm.py -m gpu -k "not c4_scale" > gpurun_out/slabs_ab_tests.log 2>&1 || { tail -30 gpurun_out/slabs_ab_tests.log; exit 1; }
tail -1 gpurun_out/slabs_ab_tests.log
for i in $(seq 1 ${ROUNDS:-3}); do
  for n in "$@"; do
    CC_LIB_PATH=$ROOT/tools/ab/lib_$n.so timeout -k 10 200 python -u tools/bench_sharded_slabs.py 8 c3 10 > gpurun_out/sab_$n.json 2> gpurun_out/sab_$n.err
    python3 -c "
import json; d=json.loads(open('gpurun_out/sab_$n.json').read().strip().splitlines()[-1])
k=d['middle_slab_kernels_ms']; print('$n', d['per_slab_ms'], d['ratio_to_ideal'], len(k), round(sum(k.values()),4), {a: k[a] for a in k if a not in ('k_pass2','k_spec')})"
  done
done
