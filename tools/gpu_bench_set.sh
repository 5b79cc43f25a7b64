#!/bin/bash
# GPU box: bench lines for the main workloads + one SQ-counter pass over k_spec; outputs in
# gpurun_out/.  Usage: gpurun -- tools/gpu_bench_set.sh TAG
set -e -o pipefail
TAG=${1:-cur}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
B="timeout -k 10 150 python -u bench.py --no-cpu-baseline"
$B > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err
$B --dither > gpurun_out/bench_c3cont_$TAG.json 2> gpurun_out/bench_c3cont_$TAG.err
$B --workload c4 > gpurun_out/bench_c4n1_$TAG.json 2> gpurun_out/bench_c4n1_$TAG.err
CC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload c4 --no-cpu-baseline --steps 5 \
    > gpurun_out/bench_c4n2gloo_$TAG.json 2> gpurun_out/bench_c4n2gloo_$TAG.err
tools/pmc_bench.sh pmc_spec_$TAG
python3 tools/pmc_table.py gpurun_out/pmc_spec_$TAG > gpurun_out/pmc_spec_$TAG.txt
for f in c3 c3cont c4n1 c4n2gloo; do python3 -c "
import json,sys; d=json.loads(open('gpurun_out/bench_${f}_$TAG.json').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['e2e_roofline']['frac'], d['result'].get('n_relabelled_tiles'), d['kernels_ms_per_step'])"; done
cat gpurun_out/pmc_spec_$TAG.txt
