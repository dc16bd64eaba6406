#!/bin/bash
# Round 5: full GPU suite + smoke + 1-GPU bench on the current tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5x_gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; grep -E "FAILED|^E |Error" gpurun_out/r5x_gpu_tests.log | head -30; tail -5 gpurun_out/r5x_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r5x_gpu_tests.log
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5x_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r5x_smoke.log; exit 1; }
tail -1 gpurun_out/r5x_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r5x_bench.json 2> gpurun_out/r5x_bench.err || { echo "bench failed"; tail -20 gpurun_out/r5x_bench.err; exit 1; }
cat gpurun_out/r5x_bench.json
