#!/bin/bash
# Full ALS / GBT BASELINE configs at N=1 (tools/bench_configs.py), then rocprofv3 stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/cfg_als.json > gpurun_out/cfg_als.log 2>&1 || { echo "als failed"; tail -30 gpurun_out/cfg_als.log; exit 1; }
cat gpurun_out/cfg_als.json
timeout -k 10 420 python -u tools/bench_configs.py --config gbt --trees 5 --out gpurun_out/cfg_gbt.json > gpurun_out/cfg_gbt.log 2>&1 || { echo "gbt failed"; tail -30 gpurun_out/cfg_gbt.log; exit 1; }
cat gpurun_out/cfg_gbt.json
