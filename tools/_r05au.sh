set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/sd_bench_r05au.json 2> gpurun_out/sd_bench_r05au.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload c4 --steps 10 --warmup 3 > gpurun_out/sd_bench_c4_r05au.json 2> gpurun_out/sd_bench_c4_r05au.err
python3 - <<'PY'
import json
for f in ("gpurun_out/sd_bench_r05au.json", "gpurun_out/sd_bench_c4_r05au.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d["kernels_ms_per_step"]
    print(f, "step", d["ms_per_step"], {n: v for n, v in k.items() if n.startswith("k_spec")})
PY
timeout -k 10 300 tools/roof 1024 2048 2048 5 > gpurun_out/roof_r05au.txt 2>&1
grep "mix_\|side_\|epoch_\|mask_\|rd_tile4_nt\|wr_tile " gpurun_out/roof_r05au.txt | grep "#"
