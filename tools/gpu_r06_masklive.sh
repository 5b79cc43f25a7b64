set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mask_live.py > gpurun_out/masklive_tests.log 2>&1 || { tail -40 gpurun_out/masklive_tests.log; exit 1; }
tail -1 gpurun_out/masklive_tests.log
bash tools/gpu_r06_ab.sh 39761e2 masklive "c4 c3"
