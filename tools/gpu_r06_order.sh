# k_pass2 tile order on the C3 step (CC_PASS2_ORDER), round-robin on one box; usage: tools/gpu_r06_order.sh "0 1 4" [workload]
set -e -o pipefail
mkdir -p gpurun_out
W=${2:-c3}
for i in 1 2 3; do
  for o in $1; do
    CC_PASS2_ORDER=$o timeout -k 10 150 python -u bench.py --no-cpu-baseline --workload $W --steps 10 > gpurun_out/ord_$o.json 2> gpurun_out/ord_$o.err
    python3 -c "
import json; d=json.loads(open('gpurun_out/ord_$o.json').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print('order $o', d['ms_per_step'], k['k_pass2'], k['k_spec'])"
  done
done
