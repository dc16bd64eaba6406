#!/bin/bash
# Round 5: vector tree-binning kernel: tree GPU tests, GBT full config (cold / warm, peak) + phases.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 400 $T tests/test_trees.py tests/test_gpu_estimators.py > gpurun_out/r5l_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r5l_tests.log | head -30; tail -3 gpurun_out/r5l_tests.log; exit 1; }
tail -1 gpurun_out/r5l_tests.log
timeout -k 10 400 python -u tools/bench_configs.py --config gbt --repeat 2 --out gpurun_out/r5l_cfg_gbt.json > gpurun_out/r5l_cfg_gbt.log 2>&1 \
  || { echo "gbt cfg failed"; tail -20 gpurun_out/r5l_cfg_gbt.log; exit 1; }
cut -c1-900 gpurun_out/r5l_cfg_gbt.json
timeout -k 10 400 python -u tools/bench_configs.py --config gbt --repeat 2 --trace --out gpurun_out/r5l_cfg_gbt_traced.json > gpurun_out/r5l_cfg_gbt_traced.log 2>&1 \
  || { echo "gbt traced failed"; tail -20 gpurun_out/r5l_cfg_gbt_traced.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5l_cfg_gbt_traced.json')); print(d['value'], d.get('fit_seconds_each'), json.dumps(d.get('phases_s'))[:900])"
