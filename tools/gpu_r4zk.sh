#!/bin/bash
# Woodbury rows with 17..24 ratings in a 24-row launch (115 VGPRs; O3S_ALS_WOOD_SPLIT24=1) vs with the 32-row ones.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py \
  > gpurun_out/r4zk_tests.log 2>&1 || { echo "tests failed"; grep -E "assert|Error" gpurun_out/r4zk_tests.log | head -10; tail -5 gpurun_out/r4zk_tests.log; exit 1; }
tail -1 gpurun_out/r4zk_tests.log
for m in 0 1 0 1; do
  O3S_ALS_WOOD_SPLIT24=$m timeout -k 10 200 python -u tools/bench_als.py --rank-of 8 --users 50000000 --items 5000000 \
    --ratings 1000000000 --iters 2 > gpurun_out/r4zk_als_$m.json 2> gpurun_out/r4zk_als_$m.err \
    || { echo "bench_als $m failed"; tail -20 gpurun_out/r4zk_als_$m.err; exit 1; }
  echo "split24=$m $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4zk_als_$m.json').read().strip().splitlines()[-1]); print(d['value'])")"
done
for m in 0 1; do
O3S_ALS_WOOD_SPLIT24=$m timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --trace --out gpurun_out/r4zk_cfg_als_traced_$m.json > gpurun_out/r4zk_cfg_$m.log 2>&1 || { echo "als cfg failed"; tail -30 gpurun_out/r4zk_cfg_$m.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4zk_cfg_als_traced_$m.json')); print('split24=$m', d['value'], d['fit_seconds'], d['phases_s']['als.woodbury'])"
done
