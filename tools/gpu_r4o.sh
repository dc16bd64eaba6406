#!/bin/bash
# ALS dense kernel: 4-step LDS-DMA ring with unpadded, XOR-swizzled bf16 staging.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py \
  > gpurun_out/r4o_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4o_tests.log; exit 1; }
tail -1 gpurun_out/r4o_tests.log
timeout -k 10 200 python -u tools/als_dense_phases.py --gl 1 > gpurun_out/r4o_phases.json 2> gpurun_out/r4o_phases.err \
  || { echo "phases failed"; tail -20 gpurun_out/r4o_phases.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4o_phases.json
for v in mfma_gl mfma_blk mfma_gl; do
  O3S_ALS_DENSE=$v timeout -k 10 200 python -u tools/bench_als.py --rank-of 8 --users 50000000 --items 5000000 \
    --ratings 1000000000 --iters 2 > gpurun_out/r4o_als_$v.json 2> gpurun_out/r4o_als_$v.err \
    || { echo "bench_als $v failed"; tail -20 gpurun_out/r4o_als_$v.err; exit 1; }
  echo "$v $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4o_als_$v.json').read().strip().splitlines()[-1]); print(d['value'])")"
done
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/r4o_cfg_als.json > gpurun_out/r4o_cfg_als.log 2>&1 || { echo "als cfg failed"; tail -30 gpurun_out/r4o_cfg_als.log; exit 1; }
cat gpurun_out/r4o_cfg_als.json
