# k_pass2 occupancy sensitivity: CC_LDS_PAD_P2 bytes of extra LDS per workgroup (4 -> 3 -> 2 tiles per CU)
set -e -o pipefail
mkdir -p gpurun_out
for p in 0 12000 25000 0; do
  CC_LDS_PAD_P2=$p timeout -k 10 150 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/pad_$p.json 2> gpurun_out/pad_$p.err
  python3 -c "
import json; d=json.loads(open('gpurun_out/pad_$p.json').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print($p, d['ms_per_step'], k['k_pass2'], k['k_spec'])"
done
