set -e -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 rocm-smi --showvbios 2>&1 | grep -i "vbios version" || true
: > gpurun_out/ab_r05ax.txt
for rep in 1 2; do
  for o in 0 1 2; do
    for wl in c2 c1; do
      CC_PASS2_ORDER=$o timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload $wl --steps 50 --warmup 5 > gpurun_out/ab_r05ax_cur.json 2>> gpurun_out/ab_r05ax.err
      python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_r05ax_cur.json').read().strip().splitlines()[-1]); print('$wl', 'order=$o', 'rep=$rep', 'step', d['ms_per_step'], 'k_pass2', d['kernels_ms_per_step']['k_pass2'])" >> gpurun_out/ab_r05ax.txt
    done
  done
done
cat gpurun_out/ab_r05ax.txt
