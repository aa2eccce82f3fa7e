#!/bin/bash
# One GPU-box call of a round's measurements (rounds 5-6): the steps named on the command
# line, in order, each under its own time limit, stopping at the first failure.
#   bash tools/gpu_round.sh TAG step...
# steps:
#   pytest     the whole -m gpu suite
#   fused      the fused-combine / config-size GPU tests only
#   classify   tools/classify_cost (pointer kinds: HSA vs HIP query)
#   fold       tools/fold_trace (fused fold workgroup trace + candidate shapes)
#   local      tools/local_ranks_ab.py (8 concurrent host-combine ranks)
#   smoke      __graft_entry__.smoke()
#   bench      python bench.py (defaults)
#   prof       tools/profile_r03.sh: kernel trace + stats at 256 / 64 MiB, FETCH_SIZE and WRITE_SIZE passes
#   lds        tools/archive/lds_cap_cost (a fused fold beside a streaming kernel)
#   hostlat    tools/host_small_latency gpu
#   driver6    python bench.py --steps 20 --warmup 5 (the driver's shape), six fresh processes
#   bench20    python bench.py --steps 20 --warmup 5, once (round 6: one bench pass per product change)
#   classifyt  tests/test_classify_kinds_gpu.py (pointer kinds, kept verdicts)
#   bindt      tests/test_bind_gpu.py (the binding and signal-node knobs)
#   place      tools/placement_ab.py (near / far / as-launched caller, alternated processes)
#   place2     the same with the waiting knobs (lazy / delay / flush polls) beside near and far
#   place3     near / far callers with the completion signal on the GPU's node (sigg) or another (sigo)
#   cpfloor    tools/aql/cp_floor.sh (the CP's doorbell -> start floor with HSA alone, then the product's split)
#   ccd        tools/archive/ccd_ab.py (the calling thread moved across L3 domains in one process)
#   pairalloc  tools/archive/pair_alloc_ab.py --ab (per-pair call and kernel medians under four allocation methods)
#   pipe       the collectives' GPU tests (loopback, config sizes, fused schedules)
#   overlap    tools/archive/pipeline_overlap (fold beside a one-rank RCCL transfer, serial vs overlapped, capped or not)
#   pipeab     tools/archive/pipeline_ab.py (config 5 through the loopback, pipelined vs not)
#   overhead   tools/archive/timing_overhead.py (the timed region's bracketing cost; raw profiled splits), near and unbound
#   share2     BENCH_TEST_SHARE_GPU=1 bench.py --gpus 2 (the N > 1 path rehearsed on one GPU; not a measurement)
#   rotate     tools/archive/fold_rotate (P = 8 fold with rotated operand reads)
# Build every binary on the CPU side first (make -C mpich-pip_amd; hipcc lines
# in each tool's header).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
    echo "== $step $(date +%T)"
    case $step in
    pytest) timeout -k 10 420 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/ \
                > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -2 $OUT/pytest_gpu.log ;;
    fused) timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
                tests/test_schedule_fused_gpu.py tests/test_coll_loopback_gpu.py tests/test_config_size_gpu.py \
                > $OUT/pytest_fused.log 2>&1; rc=$?; tail -2 $OUT/pytest_fused.log ;;
    classify) timeout -k 10 120 tools/classify_cost > $OUT/classify_cost.log 2>&1; rc=$?; cat $OUT/classify_cost.log ;;
    fold) timeout -k 10 400 tools/fold_trace > $OUT/fold_trace.log 2>&1; rc=$?; cat $OUT/fold_trace.log ;;
    local) timeout -k 10 400 python -u tools/local_ranks_ab.py 5 > $OUT/local_ranks_ab.log 2>&1; rc=$?
           cat $OUT/local_ranks_ab.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
           tail -5 $OUT/smoke.log ;;
    bench) timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1; rc=$?; tail -c 3000 $OUT/bench.log ;;
    prof) timeout -k 10 1100 bash tools/profile_r03.sh $TAG > $OUT/prof.log 2>&1; rc=$?; tail -3 $OUT/prof.log ;;
    lds) timeout -k 10 300 tools/archive/lds_cap_cost > $OUT/lds_cap_cost.log 2>&1; rc=$?; cat $OUT/lds_cap_cost.log ;;
    hostlat) timeout -k 10 200 tools/host_small_latency gpu > $OUT/host_small_latency.log 2>&1; rc=$?
             cat $OUT/host_small_latency.log ;;
    driver6) rc=0
             for i in 1 2 3 4 5 6; do
                 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_ds_$i.log 2>&1 || { rc=$?; break; }
                 python - $OUT/bench_ds_$i.log <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
c = d["call_distribution"]
print(f"{sys.argv[1]}: value {d['value']} = {d['per_gpu']['frac_of_hbm_peak']}, kernel {d['roofline']['mean_launch_us']} us "
      f"({d['roofline']['frac']}), call median {c['median_us']} p90 {c['p90_us']}, fixed {c['decomposition']['fixed_us']}")
PY
             done ;;
    bench20) timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench20.log 2>&1; rc=$?
             tail -c 3000 $OUT/bench20.log ;;
    classifyt) timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
                tests/test_classify_kinds_gpu.py > $OUT/pytest_classify.log 2>&1; rc=$?; tail -4 $OUT/pytest_classify.log ;;
    bindt) timeout -k 10 300 python -u -m pytest -x -v --timeout 180 --timeout-method thread \
                tests/test_bind_gpu.py > $OUT/pytest_bind.log 2>&1; rc=$?; tail -6 $OUT/pytest_bind.log ;;
    place) timeout -k 10 600 python -u tools/placement_ab.py 4 2000 > $OUT/placement_ab.log 2>&1; rc=$?
           tail -8 $OUT/placement_ab.log ;;
    place2) timeout -k 10 900 python -u tools/placement_ab.py 3 2000 near,far,near:lazy,far:lazy,near:flush,near:delay \
                > $OUT/placement_ab2.log 2>&1; rc=$?; tail -9 $OUT/placement_ab2.log ;;
    place3) timeout -k 10 900 python -u tools/placement_ab.py 3 2000 near,near:sigg,near:sigo,far,far:sigg,far:sigo \
              > $OUT/placement_sig.log 2>&1; rc=$?; tail -9 $OUT/placement_sig.log ;;
    cpfloor) timeout -k 10 600 bash tools/aql/cp_floor.sh > $OUT/cp_floor.log 2>&1; rc=$?; grep -v '^{' $OUT/cp_floor.log | tail -30 ;;
    ccd) timeout -k 10 300 python -u tools/archive/ccd_ab.py 20 > $OUT/ccd_ab.log 2>&1; rc=$?; grep -v '^{"round' $OUT/ccd_ab.log | tail -24 ;;
    pairalloc) timeout -k 10 600 python -u tools/archive/pair_alloc_ab.py --ab 3 > $OUT/pair_alloc_ab.log 2>&1; rc=$?; tail -6 $OUT/pair_alloc_ab.log ;;
    pipe) timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
                tests/test_coll_loopback_gpu.py tests/test_config_size_gpu.py tests/test_schedule_fused_gpu.py \
                > $OUT/pytest_pipe.log 2>&1; rc=$?; tail -2 $OUT/pytest_pipe.log ;;
    overlap) timeout -k 10 200 tools/archive/pipeline_overlap 15 > $OUT/pipeline_overlap.log 2>&1; rc=$?
             cat $OUT/pipeline_overlap.log ;;
    pipeab) timeout -k 10 300 python -u tools/archive/pipeline_ab.py 7 > $OUT/pipeline_ab.log 2>&1; rc=$?
            cat $OUT/pipeline_ab.log ;;
    overhead) { timeout -k 10 120 python3 -u tools/archive/timing_overhead.py > $OUT/overhead_near.log 2>&1 &&
                timeout -k 10 120 python3 -u tools/archive/timing_overhead.py unbound > $OUT/overhead_none.log 2>&1; }; rc=$?
              cat $OUT/overhead_near.log $OUT/overhead_none.log ;;
    share2) BENCH_TEST_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --mib 64 --steps 10 --warmup 3 \
                --collectives off > $OUT/bench_share2.log 2>&1; rc=$?; tail -c 1500 $OUT/bench_share2.log ;;
    rotate) timeout -k 10 400 tools/archive/fold_rotate 9 > $OUT/fold_rotate.log 2>&1; rc=$?; cat $OUT/fold_rotate.log ;;
    *) echo "unknown step $step"; rc=2 ;;
    esac
    if [ $rc -ne 0 ]; then echo "step $step failed: $rc"; exit $rc; fi
done
