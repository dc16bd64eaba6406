#!/bin/bash
# Kernel stats of the full ALS config after the round-4 kernel work.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r4t_prof_als" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --config als --iters 3) \
  > gpurun_out/r4t_prof_als.log 2>&1 || { echo "als profile failed"; tail -20 gpurun_out/r4t_prof_als.log; exit 1; }
head -25 gpurun_out/r4t_prof_als/run_kernel_stats.csv | cut -c1-120
