set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 python3 tools/kfd_probe.py > gpurun_out/kfd_probe.log 2>&1
timeout -k 10 60 tools/host_small_latency > gpurun_out/host_small_latency.log 2>&1
timeout -k 10 60 tools/host_small_latency gpu > gpurun_out/host_small_latency_gpu.log 2>&1
timeout -k 10 200 python -u -m pytest tests/test_host_only_gpu.py tests/test_direct_prepare_gpu.py tests/test_host_only_cpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r04a.log 2>&1 && \
timeout -k 10 400 python3 tools/ring_placement_ab.py 4 > gpurun_out/ring_placement_ab.log 2>&1
rc=$?
cat gpurun_out/kfd_probe.log gpurun_out/host_small_latency*.log; tail -5 gpurun_out/pytest_r04a.log; tail -3 gpurun_out/ring_placement_ab.log
exit $rc
