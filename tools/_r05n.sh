set -e -o pipefail
tools/gpu_steps.sh r05n boxinfo roof bench_full bench_c4 bench_c2 bench_c1 bench_cont slabs8_c3 slabs8_c4
