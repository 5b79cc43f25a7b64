#!/bin/bash
# One GPU-box session of named evidence steps, run in order; each GPU step has its own time
# limit and the session stops at the first failure (no retries).  Outputs under gpurun_out/.
# Usage (from this container): gpurun --timeout 1200 -- tools/gpu_steps.sh TAG STEP [STEP ...]
#   bench          default bench line (C3, N = 1), CPU baseline skipped    -> bench_TAG.json
#   bench_full     default bench line with the CPU baseline                 -> bench_full_TAG.json
#   bench_c4 / bench_c2 / bench_c1 / bench_cont   other workloads on one GPU
#   slabs8_c3 / slabs8_c4   the 8-slab strong-scaling schedule in one process (tools/bench_sharded_slabs.py)
#   n2gloo / n4gloo  bench.py --gpus 2 --workload c4 / --gpus 4 --workload c3 self-launched, gloo on one GPU
#   tests          the whole -m gpu suite                                   -> tests_TAG.log
#   smoke          __graft_entry__.smoke()                                  -> smoke_TAG.log
#   tests_comm     the sharded C entry: world 1 on RCCL, world 2 / 3 on the test-only stand-in
#   bench_c5       one rank's C5 slab (256, 4096, 4096)
#   c1_dropin      BASELINE C1 through ThresholdedComponentsWorkflow, per-stage job wall (tools/bench_c1.py)
#   tests_workflow tests/test_gpu_workflow.py
#   tests_sharded  tests/test_gpu_sharded.py only;  tests_parity  parity + watershed + workflow files
#   bench_sync / bench_c2_sync   the host-synchronised schedule (CC_FAST=0), same-box A/B
#   prof_c3 / prof_c3_mask / prof_cont / prof_c2 / prof_c1   rocprofv3 trace + FETCH/WRITE passes (tools/profile.sh)
#   trace_slabs8   rocprofv3 kernel trace of the 8-slab schedule
#   evidence       rocprof summaries of the secondary kernels (threshold, stage path, 8-slab seams of
#                  both schedules, Gaussian prefilter, resized mask + 4-D normalize, watershed);  prof_c4  C3 + mask with the --narrow correction
#   clock          effective GPU clock per kernel of the C3 step (tools/pmc_clock.sh)
#   roof / ablate  the box's streaming ceilings (tools/roof) and the k_spec ablation (tools/ablate)
#   ab_fast        same-box round-robin A/B: one-read-back vs host-synchronised schedule (C3)
#   boxinfo        the lease's static / current SMI info (product, VBIOS, power cap, clocks, memory)
#   clockprobe     core clock per kernel from in-kernel clock stamps (tools/clock_probe)
#   slowdiag       a short bench first; only when k_spec runs slow (> 3.3 ms, the driver's slow box
#                  kind) the box's roof, the k_spec ablation, the clock probe and the PMC passes
#                  (TCP latency / UTCL1, SQ instruction + wait counters) -> *_slow_TAG
set -e -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
O=gpurun_out
PYT="python -u -m pytest -x -v --timeout 400 --timeout-method thread"
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    bench)      timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_$TAG.json 2> $O/bench_$TAG.err; cat $O/bench_$TAG.json ;;
    bench_full) timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_full_$TAG.json 2> $O/bench_full_$TAG.err; cat $O/bench_full_$TAG.json ;;
    bench_c4)   timeout -k 10 240 python -u bench.py --no-cpu-baseline --workload c4 --steps 20 --warmup 5 > $O/bench_c4_$TAG.json 2> $O/bench_c4_$TAG.err; cat $O/bench_c4_$TAG.json ;;
    bench_c4_sync) CC_FAST=0 timeout -k 10 240 python -u bench.py --no-cpu-baseline --workload c4 --steps 20 --warmup 5 > $O/bench_c4_sync_$TAG.json 2> $O/bench_c4_sync_$TAG.err; cat $O/bench_c4_sync_$TAG.json ;;
    bench_c1_sync) CC_FAST=0 timeout -k 10 240 python -u bench.py --no-cpu-baseline --workload c1 --steps 50 --warmup 10 > $O/bench_c1_sync_$TAG.json 2> $O/bench_c1_sync_$TAG.err; cat $O/bench_c1_sync_$TAG.json ;;
    bench_c2)   timeout -k 10 240 python -u bench.py --no-cpu-baseline --workload c2 --steps 50 --warmup 10 > $O/bench_c2_$TAG.json 2> $O/bench_c2_$TAG.err; cat $O/bench_c2_$TAG.json ;;
    bench_c1)   timeout -k 10 240 python -u bench.py --no-cpu-baseline --workload c1 --steps 50 --warmup 10 > $O/bench_c1_$TAG.json 2> $O/bench_c1_$TAG.err; cat $O/bench_c1_$TAG.json ;;
    bench_cont) timeout -k 10 240 python -u bench.py --no-cpu-baseline --dither --steps 20 --warmup 5 > $O/bench_cont_$TAG.json 2> $O/bench_cont_$TAG.err; cat $O/bench_cont_$TAG.json ;;
    bench_c2_sync) CC_FAST=0 timeout -k 10 240 python -u bench.py --no-cpu-baseline --workload c2 --steps 50 --warmup 10 > $O/bench_c2_sync_$TAG.json 2> $O/bench_c2_sync_$TAG.err; cat $O/bench_c2_sync_$TAG.json ;;
    bench_sync) CC_FAST=0 timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_sync_$TAG.json 2> $O/bench_sync_$TAG.err; cat $O/bench_sync_$TAG.json ;;
    tests_parity) timeout -k 10 900 $PYT tests/test_gpu_parity.py tests/test_watershed.py tests/test_gpu_workflow.py > $O/tests_parity_$TAG.log 2>&1 || { tail -40 $O/tests_parity_$TAG.log; exit 1; }; tail -3 $O/tests_parity_$TAG.log ;;
    slabs8_c3)  timeout -k 10 300 python -u tools/bench_sharded_slabs.py 8 c3 10 > $O/slabs8_c3_$TAG.json 2> $O/slabs8_c3_$TAG.err; cat $O/slabs8_c3_$TAG.json ;;
    slabs8_c4)  timeout -k 10 300 python -u tools/bench_sharded_slabs.py 8 c4 10 > $O/slabs8_c4_$TAG.json 2> $O/slabs8_c4_$TAG.err; cat $O/slabs8_c4_$TAG.json ;;
    n4gloo)     CC_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 4 --workload c3 --steps 5 --warmup 2 --no-cpu-baseline > $O/n4gloo_$TAG.json 2> $O/n4gloo_$TAG.err; cat $O/n4gloo_$TAG.json ;;
    n2gloo)     CC_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > $O/n2gloo_$TAG.json 2> $O/n2gloo_$TAG.err; cat $O/n2gloo_$TAG.json ;;
    tests)      timeout -k 10 1000 $PYT tests -m gpu > $O/tests_$TAG.log 2>&1 || { tail -40 $O/tests_$TAG.log; exit 1; }; tail -3 $O/tests_$TAG.log ;;
    smoke)      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { tail -20 $O/smoke_$TAG.log; exit 1; }; tail -3 $O/smoke_$TAG.log ;;
    tests_comm) timeout -k 10 600 $PYT tests/test_gpu_comm.py tests/test_gpu_comm_ranks.py > $O/tests_comm_$TAG.log 2>&1 || { tail -40 $O/tests_comm_$TAG.log; exit 1; }; tail -3 $O/tests_comm_$TAG.log ;;
    bench_c5)   timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload c5 --steps 20 --warmup 5 > $O/bench_c5_$TAG.json 2> $O/bench_c5_$TAG.err; cat $O/bench_c5_$TAG.json ;;
    c1_dropin)  timeout -k 10 600 python -u tools/bench_c1.py --repeats 3 > $O/c1_dropin_$TAG.json 2> $O/c1_dropin_$TAG.err; cat $O/c1_dropin_$TAG.json ;;
    tests_workflow) timeout -k 10 900 $PYT tests/test_gpu_workflow.py > $O/tests_workflow_$TAG.log 2>&1 || { tail -40 $O/tests_workflow_$TAG.log; exit 1; }; tail -3 $O/tests_workflow_$TAG.log ;;
    tests_sharded) timeout -k 10 900 $PYT tests/test_gpu_sharded.py > $O/tests_sharded_$TAG.log 2>&1 || { tail -40 $O/tests_sharded_$TAG.log; exit 1; }; tail -3 $O/tests_sharded_$TAG.log ;;
    prof_c3)    tools/profile.sh "${TAG}_c3" --steps 10 --warmup 3 ;;
    prof_c3_mask) tools/profile.sh "${TAG}_c3_mask" --steps 10 --warmup 3 --mask ;;
    prof_cont)  tools/profile.sh "${TAG}_c3_cont" --steps 10 --warmup 3 --dither ;;
    prof_c2)    tools/profile.sh "${TAG}_c2" --workload c2 --steps 20 --warmup 5 ;;
    prof_c1)    tools/profile.sh "${TAG}_c1" --workload c1 --steps 20 --warmup 5 ;;
    evidence)   # rocprof trace + FETCH / WRITE of the secondary kernels (tools/profile_cmd.sh)
                P=tools/profile_cmd.sh
                $P ${TAG}_threshold tools/bench_threshold.py
                $P ${TAG}_stage tools/bench_stage.py
                $P ${TAG}_slabs8 tools/bench_sharded_slabs.py 8 c3 3
                $P ${TAG}_prefilter tools/bench_prefilter.py --steps 3
                NARROW=k_mask_resize=536870912 $P ${TAG}_misc tools/bench_misc.py
                $P ${TAG}_slabs8sync tools/bench_sharded_slabs.py 8 c3 2 sync
                $P ${TAG}_watershed tools/bench_watershed.py ;;
    prof_c4)    CC_NVOX=4294967296 tools/profile.sh "${TAG}_c4" --workload c4 --steps 10 --warmup 3 --mask ;;
    ab_fast)    ROUNDS=3 timeout -k 10 600 tools/gpu_ab.sh "CC_FAST=1" "CC_FAST=0" > $O/ab_fast_$TAG.txt 2>&1; cat $O/ab_fast_$TAG.txt ;;
    clock)      tools/pmc_clock.sh "$TAG" ;;
    roof)       timeout -k 10 300 tools/roof 1024 2048 2048 5 > $O/roof_$TAG.txt 2>&1; tail -40 $O/roof_$TAG.txt ;;
    ablate)     timeout -k 10 300 tools/ablate 1024 2048 2048 64 512 512 0 10 > $O/ablate_$TAG.txt 2>&1; tail -5 $O/ablate_$TAG.txt ;;
    trace_slabs8) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
                    -d "$ROOT/$O/trace_slabs8_$TAG" -o run -- python3 "$ROOT/tools/bench_sharded_slabs.py" 8 c3 3 \
                    > "$ROOT/$O/trace_slabs8_$TAG.json" 2> "$ROOT/$O/trace_slabs8_$TAG.err") ;;
    boxinfo)    { timeout -k 5 60 rocm-smi --showproductname --showvbios --showdriverversion --showpower --showmaxpower \
                    --showclocks --showmemvendor --showmeminfo vram --showcomputepartition --showmemorypartition 2>&1 || true;
                  timeout -k 5 60 amd-smi static -g 0 2>&1 || true; timeout -k 5 60 amd-smi metric -g 0 2>&1 || true; } > $O/boxinfo_$TAG.txt
                grep -iE "vbios|power cap|max.*power|sclk|mclk|fclk|partition|Card Series|Market" $O/boxinfo_$TAG.txt | head -40 || true ;;
    clockprobe) timeout -k 10 120 tools/clock_probe 1024 2048 2048 64 512 512 4 > $O/clockprobe_$TAG.txt 2>&1; cat $O/clockprobe_$TAG.txt ;;
    slowdiag)   timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/sd_bench_$TAG.json 2> $O/sd_bench_$TAG.err
                KS=$(python3 -c "import json; d = json.loads(open('$O/sd_bench_$TAG.json').read().strip().splitlines()[-1]); print(d['kernels_ms_per_step']['k_spec'])")
                echo "k_spec $KS ms"
                if python3 -c "import sys; sys.exit(0 if $KS > 3.3 else 1)"; then
                  echo "slow box kind: diagnostics"
                  timeout -k 10 300 tools/roof 1024 2048 2048 5 > $O/roof_slow_$TAG.txt 2>&1
                  timeout -k 10 300 tools/ablate 1024 2048 2048 64 512 512 0 10 > $O/ablate_slow_$TAG.txt 2>&1
                  timeout -k 10 120 tools/clock_probe 1024 2048 2048 64 512 512 4 > $O/clockprobe_slow_$TAG.txt 2>&1
                  tools/pmc_tcp.sh && mv $O/pmc_tcp $O/pmc_tcp_slow_$TAG
                  tools/pmc_ablate.sh pmc_ablate_slow_$TAG 1024 2048 2048 64 512 512 0
                  tail -3 $O/ablate_slow_$TAG.txt; grep -E "k_spec|k_pass2" $O/clockprobe_slow_$TAG.txt | head -4
                else
                  echo "fast box kind: no diagnostics"
                fi ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
