#!/bin/bash
# Round-4 GPU batch B: ALS dense-kernel correctness + A/B (mfma_blk vs mfma_pf), pool ALS,
# GBT histogram PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py \
  > gpurun_out/r4b_als_tests.log 2>&1 || { echo "als tests failed"; tail -40 gpurun_out/r4b_als_tests.log; exit 1; }
tail -2 gpurun_out/r4b_als_tests.log
for k in mfma_blk mfma_pf mfma_blk mfma_pf; do
  O3S_ALS_DENSE=$k timeout -k 10 200 python -u tools/bench_als.py --rank-of 8 --users 50000000 --items 5000000 \
    --ratings 1000000000 --iters 2 > gpurun_out/r4b_als_$k.json 2> gpurun_out/r4b_als_$k.err \
    || { echo "bench_als $k failed"; tail -20 gpurun_out/r4b_als_$k.err; exit 1; }
  echo "$k $(cat gpurun_out/r4b_als_$k.json)"
done
timeout -k 10 420 python -u tools/bench_pool_als.py > gpurun_out/r4b_pool_als.log 2>&1 || { echo "pool als failed"; tail -30 gpurun_out/r4b_pool_als.log; exit 1; }
tail -1 gpurun_out/r4b_pool_als.log
timeout -k 10 600 bash tools/pmc_gbt_hist.sh || { echo "pmc gbt failed"; exit 1; }
cat gpurun_out/pmc_gbt/summary.txt
# kernel stats of the full ALS / GBT configs (fit through the estimator API)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg_als" \
   -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --config als --iters 2) > gpurun_out/prof_cfg_als.log 2>&1 \
   || { echo "prof als failed"; tail -20 gpurun_out/prof_cfg_als.log; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg_gbt" \
   -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --config gbt --trees 3) > gpurun_out/prof_cfg_gbt.log 2>&1 \
   || { echo "prof gbt failed"; tail -20 gpurun_out/prof_cfg_gbt.log; exit 1; }
echo profiled
