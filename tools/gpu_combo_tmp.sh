#!/bin/bash
set -e -o pipefail
cd ${GRAFT_REPO_ROOT}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread -k "stage or large or faces or write or sharded" > gpurun_out/tests_st2.log 2>&1 || { tail -40 gpurun_out/tests_st2.log; exit 1; }
tail -2 gpurun_out/tests_st2.log
timeout -k 10 300 python -u tools/bench_stage.py greater > gpurun_out/stage_st2.json && cat gpurun_out/stage_st2.json
ROUNDS=3 tools/gpu_ab_libs.sh base wl prefetch pfwl
