#!/bin/bash
# SQ instruction / wait counters per kernel variant of tools/ablate (one PMC pass).
# Usage: tools/pmc_ablate.sh OUTDIR Z Y X bz by bx mode
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES \
    --output-format csv -d "$OUT" -o run -- "$ROOT/tools/ablate" "$@" 1 > /dev/null 2>&1
