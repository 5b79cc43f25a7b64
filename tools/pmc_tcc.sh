#!/bin/bash
# L2 -> memory (TCC_EA) request / stall counters per kernel variant of tools/ablate, two passes of
# at most 4 TCC counters each (MI355X_MICROARCH.md: no counter splitting across passes).
# Usage: tools/pmc_tcc.sh OUTDIR   -> gpurun_out/OUTDIR/{p1,p2}
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$1
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
grep -o "TCC_EA0_[A-Z_]*" "$OUT/avail.txt" | sort -u > "$OUT/tcc_ea.txt" || true
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d "$OUT/p1" -o run -- "$ROOT/tools/ablate" 1024 2048 2048 64 512 512 0 1 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_STALL_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d "$OUT/p2" -o run -- "$ROOT/tools/ablate" 1024 2048 2048 64 512 512 0 1 > /dev/null 2>&1
