#!/bin/bash
# Round-4 GPU batch E: ALS dense-kernel locality probe (gather table 1M vs 50M rows) + PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py \
  > gpurun_out/r4e_als_tests.log 2>&1 || { echo "als tests failed"; tail -40 gpurun_out/r4e_als_tests.log; exit 1; }
tail -1 gpurun_out/r4e_als_tests.log
for k in mfma_blk mfma_dp mfma_blk mfma_dp; do
  O3S_ALS_DENSE=$k timeout -k 10 200 python -u tools/bench_als.py --rank-of 8 --users 50000000 --items 5000000 \
    --ratings 1000000000 --iters 2 > gpurun_out/r4e_als_$k.json 2> gpurun_out/r4e_als_$k.err \
    || { echo "bench_als $k failed"; tail -20 gpurun_out/r4e_als_$k.err; exit 1; }
  echo "$k $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4e_als_$k.json').read().strip().splitlines()[-1]); print(d['value'])")"
done
for other in 1000000 8000000 50000000; do
  timeout -k 10 240 python -u tools/prof_als_exact.py --users 2000000 --items 625000 --other $other --other-item $other --reps 2 \
    > gpurun_out/r4e_als_other_$other.log 2>&1 || { echo "prof_als $other failed"; tail -20 gpurun_out/r4e_als_other_$other.log; exit 1; }
  echo "other=$other $(grep -E '^(user|item)' gpurun_out/r4e_als_other_$other.log | tr '\n' ' ')"
done
timeout -k 10 600 bash tools/pmc_als_exact.sh || { echo "pmc als failed"; exit 1; }
cat gpurun_out/pmc_als/summary_dense.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_trees.py \
  > gpurun_out/r4e_tree_tests.log 2>&1 || { echo "tree tests failed"; tail -30 gpurun_out/r4e_tree_tests.log; exit 1; }
O3S_HIST_WIDE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_trees.py \
  > gpurun_out/r4e_tree_tests_wide.log 2>&1 || { echo "tree tests (wide) failed"; tail -30 gpurun_out/r4e_tree_tests_wide.log; exit 1; }
tail -1 gpurun_out/r4e_tree_tests_wide.log
for wide in 0 1 0 1; do
  O3S_HIST_WIDE=$wide timeout -k 10 200 python -u tools/bench_gbt.py --trees 3 > gpurun_out/r4e_gbt_w$wide.json 2> gpurun_out/r4e_gbt_w$wide.err \
    || { echo "bench_gbt $wide failed"; tail -20 gpurun_out/r4e_gbt_w$wide.err; exit 1; }
  echo "wide=$wide $(python3 -c "import json; d=json.loads(open('gpurun_out/r4e_gbt_w$wide.json').read().strip().splitlines()[-1]); print(d['value'], d['loss'][-1])")"
done
