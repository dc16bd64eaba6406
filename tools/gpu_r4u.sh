#!/bin/bash
# x = Q y on the matrix cores (O3S_ALS_ROTATE_MFMA=1) vs the packed-FMA rotate kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
O3S_ALS_ROTATE_MFMA=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py \
  > gpurun_out/r4u_tests.log 2>&1 || { echo "tests failed"; grep -E "assert|Error" gpurun_out/r4u_tests.log | head -10; tail -5 gpurun_out/r4u_tests.log; exit 1; }
tail -1 gpurun_out/r4u_tests.log
for m in 0 1 0 1; do
  O3S_ALS_ROTATE_MFMA=$m timeout -k 10 200 python -u tools/bench_als.py --rank-of 8 --users 50000000 --items 5000000 \
    --ratings 1000000000 --iters 2 > gpurun_out/r4u_als_$m.json 2> gpurun_out/r4u_als_$m.err \
    || { echo "bench_als $m failed"; tail -20 gpurun_out/r4u_als_$m.err; exit 1; }
  echo "rot_mfma=$m $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4u_als_$m.json').read().strip().splitlines()[-1]); print(d['value'])")"
done
O3S_ALS_ROTATE_MFMA=1 timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/r4u_cfg_als.json > gpurun_out/r4u_cfg_als.log 2>&1 || { echo "als cfg failed"; tail -30 gpurun_out/r4u_cfg_als.log; exit 1; }
cat gpurun_out/r4u_cfg_als.json
