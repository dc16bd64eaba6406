#!/bin/bash
# Woodbury ALS kernel: readlane-broadcast Cholesky with the forward solve fused, bucketed
# branch-free steps; 3 vs 4 waves per SIMD.  Tests, phases, rank-of-8 iteration A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py \
  > gpurun_out/r4l_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4l_tests.log; exit 1; }
tail -1 gpurun_out/r4l_tests.log
O3S_ALS_WOOD_OCC=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py -k "wood or exact" \
  > gpurun_out/r4l_tests4.log 2>&1 || { echo "occ4 tests failed"; tail -40 gpurun_out/r4l_tests4.log; exit 1; }
tail -1 gpurun_out/r4l_tests4.log
timeout -k 10 200 python -u tools/als_wood_phases.py > gpurun_out/r4l_wood_phases.json 2> gpurun_out/r4l_wood.err \
  || { echo "wood phases failed"; tail -20 gpurun_out/r4l_wood.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4l_wood_phases.json
for o in 3 4 3 4; do
  O3S_ALS_WOOD_OCC=$o timeout -k 10 200 python -u tools/bench_als.py --rank-of 8 --users 50000000 --items 5000000 \
    --ratings 1000000000 --iters 2 > gpurun_out/r4l_als_$o.json 2> gpurun_out/r4l_als_$o.err \
    || { echo "bench_als $o failed"; tail -20 gpurun_out/r4l_als_$o.err; exit 1; }
  echo "occ $o $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4l_als_$o.json').read().strip().splitlines()[-1]); print(d['value'])")"
done
timeout -k 10 240 python -u tools/prof_als_exact.py --users 2000000 --items 625000 --other 5000000 --other-item 8000000 --reps 2 \
  > gpurun_out/r4l_als_exact.log 2>&1 || { echo "prof_als failed"; tail -20 gpurun_out/r4l_als_exact.log; exit 1; }
grep -E '^(user|item)' gpurun_out/r4l_als_exact.log
