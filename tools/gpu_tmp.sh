set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_sigma.py tests/test_channel.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_sigma.log 2>&1; rc=$?; tail -30 gpurun_out/tests_sigma.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/ablate 1024 2048 2048 64 512 512 0 10 > gpurun_out/ablate_r02.txt 2>&1; cat gpurun_out/ablate_r02.txt
