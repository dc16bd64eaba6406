#!/bin/bash
# Round-4 GPU batch C: pool ALS vs in-process, GBT histogram PMC, full-config kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u tools/bench_pool_als.py > gpurun_out/r4c_pool_als.log 2>&1 || { echo "pool als failed"; tail -30 gpurun_out/r4c_pool_als.log; exit 1; }
tail -1 gpurun_out/r4c_pool_als.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg_als" \
   -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --config als --iters 2) > gpurun_out/prof_cfg_als.log 2>&1 \
   || { echo "prof als failed"; tail -20 gpurun_out/prof_cfg_als.log; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg_gbt" \
   -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --config gbt --trees 3) > gpurun_out/prof_cfg_gbt.log 2>&1 \
   || { echo "prof gbt failed"; tail -20 gpurun_out/prof_cfg_gbt.log; exit 1; }
echo profiled
timeout -k 10 600 bash tools/pmc_gbt_hist.sh || { echo "pmc gbt failed"; exit 1; }
cat gpurun_out/pmc_gbt/summary.txt
