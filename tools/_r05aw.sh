set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/suite_r05aw.txt 2>&1
tail -3 gpurun_out/suite_r05aw.txt
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r05aw.txt 2>&1
tail -1 gpurun_out/smoke_r05aw.txt
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r05aw.json 2> gpurun_out/bench_r05aw.err
tail -1 gpurun_out/bench_r05aw.json | cut -c1-400
