set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/sd_bench_r05an.json 2> gpurun_out/sd_bench_r05an.err
python3 -c "import json; d=json.loads(open('gpurun_out/sd_bench_r05an.json').read().strip().splitlines()[-1]); print('k_spec', d['kernels_ms_per_step']['k_spec'])"
tools/pmc_tcc.sh pmc_tcc_r05an
head -30 gpurun_out/pmc_tcc_r05an/tcc_ea.txt
ls gpurun_out/pmc_tcc_r05an/p1 gpurun_out/pmc_tcc_r05an/p2 | head
