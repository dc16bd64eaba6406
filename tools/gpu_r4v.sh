#!/bin/bash
# Verification of the round-4 defaults: the whole GPU suite, smoke(), the N=1 bench and its
# kernel stats, the 2-rank rehearsal of the multi-GPU bench path.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r4v_gputests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/r4v_gputests.log | head -20; tail -20 gpurun_out/r4v_gputests.log; exit 1; }
tail -1 gpurun_out/r4v_gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4v_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4v_smoke.log; exit 1; }
tail -1 gpurun_out/r4v_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r4v_bench.json 2> gpurun_out/r4v_bench.err || { echo "bench failed"; tail -20 gpurun_out/r4v_bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4v_bench.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r4v_prof_bench" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2) \
  > gpurun_out/r4v_prof_bench.log 2>&1 || { echo "bench profile failed"; tail -20 gpurun_out/r4v_prof_bench.log; exit 1; }
head -4 gpurun_out/r4v_prof_bench/run_kernel_stats.csv | cut -c1-120
timeout -k 10 600 bash tools/gpu_dist_rehearsal.sh || { echo "rehearsal failed"; exit 1; }
