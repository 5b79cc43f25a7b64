"""dev: compare per-kernel times of two bench lines (JSON files given as arguments)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d['kernels_ms_per_step']
    print(f, d['ms_per_step'], k['k_pass2'], k['k_spec'], k['k_seams'])
