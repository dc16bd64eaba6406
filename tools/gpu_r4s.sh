#!/bin/bash
# ALS Gram F^T F on the matrix cores (ftf_kernel): tests, micro-benchmark, rank-of-8 and full config.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py \
  > gpurun_out/r4s_tests.log 2>&1 || { echo "tests failed"; grep -E "assert|Error" gpurun_out/r4s_tests.log | head -10; tail -5 gpurun_out/r4s_tests.log; exit 1; }
tail -1 gpurun_out/r4s_tests.log
timeout -k 10 200 python -u tools/bench_ftf.py > gpurun_out/r4s_ftf.json 2> gpurun_out/r4s_ftf.err || { echo "bench_ftf failed"; tail -10 gpurun_out/r4s_ftf.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4s_ftf.json
for k in 1 2; do
  timeout -k 10 200 python -u tools/bench_als.py --rank-of 8 --users 50000000 --items 5000000 \
    --ratings 1000000000 --iters 2 > gpurun_out/r4s_als_$k.json 2> gpurun_out/r4s_als_$k.err \
    || { echo "bench_als failed"; tail -20 gpurun_out/r4s_als_$k.err; exit 1; }
  echo "als $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4s_als_$k.json').read().strip().splitlines()[-1]); print(d['value'])")"
done
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/r4s_cfg_als.json > gpurun_out/r4s_cfg_als.log 2>&1 || { echo "als cfg failed"; tail -30 gpurun_out/r4s_cfg_als.log; exit 1; }
cat gpurun_out/r4s_cfg_als.json
