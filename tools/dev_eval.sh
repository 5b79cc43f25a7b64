cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_evaluation.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/ev_tests.log 2>&1 || { tail -40 gpurun_out/ev_tests.log; exit 1; }
tail -3 gpurun_out/ev_tests.log
timeout -k 10 200 python tools/bench_eval.py > gpurun_out/bench_eval.json 2> gpurun_out/bench_eval.err || { tail -20 gpurun_out/bench_eval.err; exit 1; }
cat gpurun_out/bench_eval.json
