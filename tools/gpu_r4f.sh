#!/bin/bash
# Round-4 GPU batch F: the whole GPU test suite, smoke(), the N=1 headline bench, the
# 2-rank rehearsal of the multi-GPU bench path (gloo on one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r4f_gputests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|error" gpurun_out/r4f_gputests.log | head -20; tail -30 gpurun_out/r4f_gputests.log; exit 1; }
tail -1 gpurun_out/r4f_gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4f_smoke.log; exit 1; }
tail -1 gpurun_out/r4f_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r4f_bench.json 2> gpurun_out/r4f_bench.err || { echo "bench failed"; tail -20 gpurun_out/r4f_bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4f_bench.json
timeout -k 10 600 bash tools/gpu_dist_rehearsal.sh || { echo "rehearsal failed"; exit 1; }
