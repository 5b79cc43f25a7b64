#!/bin/bash
# Effective GPU clock per kernel of the C3 bench step: GRBM_GUI_ACTIVE (GPU cycles while busy) in
# its own PMC pass with the kernel trace; MHz = cycles / kernel duration (tools/pmc_clock.py).
# The box-to-box spread of k_spec follows this clock.
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_clock_$1
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d "$OUT" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/bench.json" 2> "$OUT/err.txt"
python3 "$ROOT/tools/pmc_clock.py" "$OUT" | tee "$OUT/summary.txt"
