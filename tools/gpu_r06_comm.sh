set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_comm_ranks.py > gpurun_out/r06_comm_ranks.txt 2>&1
