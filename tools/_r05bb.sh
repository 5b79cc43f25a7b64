set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r05bb.txt 2>&1
tail -1 gpurun_out/smoke_r05bb.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/parity_r05bb.txt 2>&1
tail -1 gpurun_out/parity_r05bb.txt
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_r05bb.json 2> gpurun_out/bench_r05bb.err
python3 -c "import json; d=json.loads(open('gpurun_out/bench_r05bb.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['traffic_file'], d['cpu_baseline']['value'])"
