set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
: > gpurun_out/ab_r05ay.txt
for rep in 1 2; do
  for fc in 1 2 4 8; do
    CC_FRONT_CHUNKS=$fc timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ab_r05ay_cur.json 2>> gpurun_out/ab_r05ay.err
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_r05ay_cur.json').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print('front_chunks=$fc rep=$rep step', d['ms_per_step'], 'k_spec', k.get('k_spec'), 'k_seams', k.get('k_seams'), 'k_pass2', k.get('k_pass2'))" >> gpurun_out/ab_r05ay.txt
  done
done
cat gpurun_out/ab_r05ay.txt
