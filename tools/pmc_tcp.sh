#!/bin/bash
set -e
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/pmc_tcp
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum --output-format csv -d $OUT -o run -- $ROOT/tools/ablate 1024 2048 2048 64 512 512 0 1 > /dev/null 2>&1
