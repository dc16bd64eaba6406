#!/bin/bash
# ALS with the host eigendecomposition, F Q by the rotation kernel and prefix-sum row counts: GPU tests, the full config traced (per-span times,
# iteration 1 vs the steady state) and untraced.
set -o pipefail
TAG=${1:-r4z}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py \
  > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; grep -E "assert|Error" gpurun_out/${TAG}_tests.log | head -10; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --trace --out gpurun_out/${TAG}_cfg_als_traced.json > gpurun_out/${TAG}_cfg_als_traced.log 2>&1 || { echo "als traced failed"; tail -30 gpurun_out/${TAG}_cfg_als_traced.log; exit 1; }
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/${TAG}_cfg_als.json > gpurun_out/${TAG}_cfg_als.log 2>&1 || { echo "als cfg failed"; tail -30 gpurun_out/${TAG}_cfg_als.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_cfg_als.json')); print(d['value'], d['fit_seconds'], d['iter_seconds'])"
