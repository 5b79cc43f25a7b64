#!/bin/bash
# GPU box: same-box A/B of library builds in tools/ab/lib_<name>.so (bench.py honours CC_LIB_PATH):
# a quick parity subset per build first (stops at the first failure), then ROUNDS round-robin
# bench lines.  Usage: ROUNDS=3 tools/gpu_ab_libs.sh name1 name2 ... -- [bench args]
set -e -o pipefail
V=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done
[ "$1" = "--" ] && shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"; mkdir -p gpurun_out
for n in "${V[@]}"; do
  CC_LIB_PATH=$ROOT/tools/ab/lib_$n.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x \
      --timeout 120 --timeout-method thread -k "${AB_TESTS:-synthetic_vs_oracle or white_noise or max_runs or speculated}" \
      > gpurun_out/ab_tests_$n.log 2>&1 || { echo "PARITY FAIL $n"; tail -30 gpurun_out/ab_tests_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/ab_tests_$n.log)"
done
for i in $(seq 1 ${ROUNDS:-3}); do
  for n in "${V[@]}"; do
    CC_LIB_PATH=$ROOT/tools/ab/lib_$n.so timeout -k 10 150 python -u bench.py --no-cpu-baseline --steps 10 "$@" \
        > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$n.json').read().strip().splitlines()[-1])
print('$n', d['ms_per_step'], {k: v for k, v in list(d['kernels_ms_per_step'].items())[:4]})"
  done
done
