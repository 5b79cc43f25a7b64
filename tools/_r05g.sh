set -e -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_sharded.py -k "mask_vs_oracle or c3_mask or speculated or fused_path_golden or synthetic_vs_oracle or both_schedules" > gpurun_out/t_r05g.log 2>&1 || { tail -40 gpurun_out/t_r05g.log; exit 1; }
tail -2 gpurun_out/t_r05g.log
timeout -k 10 300 tools/ablate 1024 2048 2048 64 512 512 0 10 > gpurun_out/ablate_r05g.txt 2>&1
python3 -c "
import json
for l in open('gpurun_out/ablate_r05g.txt'):
    if l.startswith('{'):
        d = json.loads(l); print({k: v for k, v in d.items() if 'spec' in k or 'copy' in k})"
timeout -k 10 200 tools/clock_probe 1024 2048 2048 64 512 512 3 > gpurun_out/clockprobe_r05g.txt 2>&1
grep -E "k_spec|sequence" gpurun_out/clockprobe_r05g.txt
ROUNDS=3 timeout -k 10 400 tools/gpu_ab.sh "CC_X=0" "CC_LIB_PATH=tools/ab/lib_mnostage.so" -- --workload c4 > gpurun_out/ab_mstage_r05g.txt 2>&1
cat gpurun_out/ab_mstage_r05g.txt
