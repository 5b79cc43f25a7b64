# Same-box A/B of a library variant against the committed build: parity + sharded files with the
# variant as the tree's library, then round-robin bench lines for the given workloads.
# Usage: tools/gpu_r06_ab.sh BASE_REV VARIANT "workload ..."
set -e -o pipefail
mkdir -p gpurun_out
B=$1; V=$2; W=${3:-c3}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sharded.py -m gpu -k "not c5 and not c4_scale" > gpurun_out/par_$V.log 2>&1 || { tail -30 gpurun_out/par_$V.log; exit 1; }
tail -1 gpurun_out/par_$V.log
for w in $W; do
  ROUNDS=3 timeout -k 10 600 tools/gpu_ab_libs.sh $B $V -- --workload $w > gpurun_out/ab_${V}_$w.txt 2>&1; echo "== $w"; cat gpurun_out/ab_${V}_$w.txt
done
