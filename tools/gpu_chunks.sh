#!/bin/bash
# GPU box: C3 bench lines for several CC_FRONT_CHUNKS (k_seams of finished z-layer chunks on a
# side stream behind k_spec of the next chunk).  gpurun_out/.
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"; mkdir -p gpurun_out
for c in 1 2 4 8 16 1; do
  CC_FRONT_CHUNKS=$c timeout -k 10 150 python -u bench.py --no-cpu-baseline > gpurun_out/bench_ch$c.json 2> gpurun_out/bench_ch$c.err
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench_ch$c.json').read().strip().splitlines()[-1])
print('chunks $c', d['value'], d['ms_per_step'], {k: v for k, v in list(d['kernels_ms_per_step'].items())[:4]})"
done
