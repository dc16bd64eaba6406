#!/bin/bash
# Round-4 GPU batch: new GPU tests, full ALS / GBT configs, pool ALS, streamed GLM rate.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_spill.py tests/test_kmeans.py > gpurun_out/r4a_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4a_tests.log; exit 1; }
tail -3 gpurun_out/r4a_tests.log
timeout -k 10 360 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/cfg_als.json > gpurun_out/cfg_als.log 2>&1 || { echo "als failed"; tail -30 gpurun_out/cfg_als.log; exit 1; }
cat gpurun_out/cfg_als.json
timeout -k 10 300 python -u tools/bench_configs.py --config gbt --trees 5 --out gpurun_out/cfg_gbt.json > gpurun_out/cfg_gbt.log 2>&1 || { echo "gbt failed"; tail -30 gpurun_out/cfg_gbt.log; exit 1; }
cat gpurun_out/cfg_gbt.json
timeout -k 10 240 python -u tools/bench_streamed.py > gpurun_out/streamed.log 2>&1 || { echo "streamed failed"; tail -30 gpurun_out/streamed.log; exit 1; }
tail -1 gpurun_out/streamed.log
