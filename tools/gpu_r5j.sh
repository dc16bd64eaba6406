#!/bin/bash
# Round 5: implicit ALS in the moving eigenbasis (no per-iteration user-table rotation):
# ALS + distributed GPU tests, full config.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 500 $T tests/test_als.py tests/test_distributed_gpu.py tests/test_pool_models_recovery.py > gpurun_out/r5j_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r5j_tests.log | head -30; tail -3 gpurun_out/r5j_tests.log; exit 1; }
tail -1 gpurun_out/r5j_tests.log
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/r5j_cfg_als.json > gpurun_out/r5j_cfg_als.log 2>&1 \
  || { echo "als cfg failed"; tail -30 gpurun_out/r5j_cfg_als.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5j_cfg_als.json')); print('full config', d['value'], d['fit_seconds'], d['iter_seconds'])"
