import json
for l in open("gpurun_out/sharded3b.json"):
    d = json.loads(l); k = d["kernels_ms"]; print(d["slab"], d["total_ms_all_slabs"], k["k_pass2"], k["k_spec"])
