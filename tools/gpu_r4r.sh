#!/bin/bash
# Woodbury persistent waves with next-row metadata prefetch (O3S_ALS_WOOD_PF=1) vs one row per wave.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py \
  > gpurun_out/r4r_tests.log 2>&1 || { echo "tests failed"; grep -E "assert|Error" gpurun_out/r4r_tests.log | head -10; tail -5 gpurun_out/r4r_tests.log; exit 1; }
tail -1 gpurun_out/r4r_tests.log
O3S_ALS_WOOD_PF=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py \
  > gpurun_out/r4r_tests_pf.log 2>&1 || { echo "pf tests failed"; grep -E "assert|Error" gpurun_out/r4r_tests_pf.log | head -10; tail -5 gpurun_out/r4r_tests_pf.log; exit 1; }
tail -1 gpurun_out/r4r_tests_pf.log
for pf in 0 1 0 1; do
  timeout -k 10 200 python -u tools/als_wood_phases.py --pf $pf > gpurun_out/r4r_wood_$pf.json 2>/dev/null || { echo "wood $pf failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r4r_wood_$pf.json').read().strip().splitlines()[-1]); print('pf', $pf, round(d['production_ms'],3))"
done
for pf in 0 1 0 1; do
  O3S_ALS_WOOD_PF=$pf timeout -k 10 200 python -u tools/bench_als.py --rank-of 8 --users 50000000 --items 5000000 \
    --ratings 1000000000 --iters 2 > gpurun_out/r4r_als_$pf.json 2> gpurun_out/r4r_als_$pf.err \
    || { echo "bench_als $pf failed"; tail -20 gpurun_out/r4r_als_$pf.err; exit 1; }
  echo "als pf=$pf $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4r_als_$pf.json').read().strip().splitlines()[-1]); print(d['value'])")"
done
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --trace --out gpurun_out/r4r_cfg_als_trace.json > gpurun_out/r4r_cfg_als_trace.log 2>&1 || { echo "als cfg failed"; tail -30 gpurun_out/r4r_cfg_als_trace.log; exit 1; }
cat gpurun_out/r4r_cfg_als_trace.json
