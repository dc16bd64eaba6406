#!/bin/bash
# ALS dense kernel: gathers overlapped with the step's MFMAs (no select on loaded values,
# indices one step ahead, no scratch arrays) -- correctness + phases + rank-of-8 timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py \
  > gpurun_out/r4h_als_tests.log 2>&1 || { echo "als tests failed"; tail -40 gpurun_out/r4h_als_tests.log; exit 1; }
tail -1 gpurun_out/r4h_als_tests.log
timeout -k 10 200 python -u tools/als_dense_phases.py > gpurun_out/r4h_phases.json 2> gpurun_out/r4h_phases.err \
  || { echo "phases failed"; tail -20 gpurun_out/r4h_phases.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4h_phases.json
for k in 1 2; do
  timeout -k 10 200 python -u tools/bench_als.py --rank-of 8 --users 50000000 --items 5000000 \
    --ratings 1000000000 --iters 2 > gpurun_out/r4h_als_$k.json 2> gpurun_out/r4h_als_$k.err \
    || { echo "bench_als failed"; tail -20 gpurun_out/r4h_als_$k.err; exit 1; }
  echo "run $k $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4h_als_$k.json').read().strip().splitlines()[-1]); print(d['value'])")"
done
timeout -k 10 240 python -u tools/prof_als_exact.py --users 2000000 --items 625000 --other 8000000 --other-item 8000000 --reps 2 \
  > gpurun_out/r4h_als_other.log 2>&1 || { echo "prof_als failed"; tail -20 gpurun_out/r4h_als_other.log; exit 1; }
grep -E '^(user|item)' gpurun_out/r4h_als_other.log
# GBT histogram: order[] of chunk c+2 issued before chunk c+1's gathers, whole chunk pairs
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_trees.py \
  > gpurun_out/r4h_tree_tests.log 2>&1 || { echo "tree tests failed"; tail -30 gpurun_out/r4h_tree_tests.log; exit 1; }
tail -1 gpurun_out/r4h_tree_tests.log
for k in 1 2; do
  timeout -k 10 200 python -u tools/bench_gbt.py --trees 3 > gpurun_out/r4h_gbt_$k.json 2> gpurun_out/r4h_gbt_$k.err \
    || { echo "bench_gbt failed"; tail -20 gpurun_out/r4h_gbt_$k.err; exit 1; }
  echo "gbt $k $(python3 -c "import json; d=json.loads(open('gpurun_out/r4h_gbt_$k.json').read().strip().splitlines()[-1]); print(d['value'], d['loss'][-1])")"
done
