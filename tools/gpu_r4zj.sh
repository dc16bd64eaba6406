#!/bin/bash
# End-of-round verification after the Woodbury short-row launch: the whole GPU
# suite, smoke(), the N=1 bench, the ALS full config (untraced) and kernel stats of it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r4zj_gputests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/r4zj_gputests.log | head -20; tail -20 gpurun_out/r4zj_gputests.log; exit 1; }
tail -1 gpurun_out/r4zj_gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4zj_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4zj_smoke.log; exit 1; }
tail -1 gpurun_out/r4zj_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r4zj_bench.json 2> gpurun_out/r4zj_bench.err || { echo "bench failed"; tail -20 gpurun_out/r4zj_bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4zj_bench.json
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/r4zj_cfg_als.json > gpurun_out/r4zj_cfg_als.log 2>&1 || { echo "als cfg failed"; tail -30 gpurun_out/r4zj_cfg_als.log; exit 1; }
cat gpurun_out/r4zj_cfg_als.json
(cd /tmp && timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r4zj_prof_als" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --config als --iters 3) \
  > gpurun_out/r4zj_prof_als.log 2>&1 || { echo "als profile failed"; tail -20 gpurun_out/r4zj_prof_als.log; exit 1; }
head -6 gpurun_out/r4zj_prof_als/run_kernel_stats.csv | cut -c1-140
for i in 1 2; do
  timeout -k 10 200 python -u tools/bench_als.py --rank-of 8 --users 50000000 --items 5000000 --ratings 1000000000 --iters 2 \
    > gpurun_out/r4zj_als8_$i.json 2> gpurun_out/r4zj_als8_$i.err || { echo "bench_als failed"; tail -20 gpurun_out/r4zj_als8_$i.err; exit 1; }
  tail -1 gpurun_out/r4zj_als8_$i.json
done
