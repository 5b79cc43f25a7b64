set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/sd_bench_r05at.json 2> gpurun_out/sd_bench_r05at.err
python3 -c "import json; d=json.loads(open('gpurun_out/sd_bench_r05at.json').read().strip().splitlines()[-1]); print('k_spec', d['kernels_ms_per_step']['k_spec'], 'step', d['ms_per_step'])"
timeout -k 10 300 tools/roof 1024 2048 2048 5 > gpurun_out/roof_r05at.txt 2>&1
grep "mix_\|side_\|epoch_\|gbar_\|rd_tile4_nt\|wr_tile " gpurun_out/roof_r05at.txt | grep "#"
