set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/smoke.log; tail -c 3000 gpurun_out/bench.log; exit $rc
