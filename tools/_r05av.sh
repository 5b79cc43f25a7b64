set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
timeout -k 10 240 python -u bench.py --no-cpu-baseline --workload c2 --steps 50 --warmup 5 > gpurun_out/sd_bench_c2_r05av.json 2> gpurun_out/sd_bench_c2_r05av.err
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/sd_bench_c2_r05av.json").read().strip().splitlines()[-1])
print("c2 step", d["ms_per_step"], d["kernels_ms_per_step"])
PY
timeout -k 10 120 tools/roof 512 512 512 50 > gpurun_out/roof_c2_r05av.txt 2>&1
grep "mix_\|side_\|mask_\|rd_tile4_nt\|rd_f4\|wr_tile \|wr_u2" gpurun_out/roof_c2_r05av.txt | grep "#"
