#!/bin/bash
# GPU box: the cold-start probes (tools/cold_probe.py, bench.py --workload c1) into gpurun_out/cold_TAG/
# Usage: gpurun -- tools/gpu_r03_cold.sh TAG
set -e -o pipefail
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
O=gpurun_out/cold_$TAG
mkdir -p $O
timeout -k 10 120 python -u tools/cold_probe.py > $O/probe.json; cat $O/probe.json
timeout -k 10 120 python -u tools/cold_probe.py > $O/probe2.json; cat $O/probe2.json
timeout -k 10 200 python -u bench.py --workload c1 > $O/c1_cold.json; cat $O/c1_cold.json
