#!/bin/bash
# ALS dense glds ring + KMeans no-distance screen: correctness, then A/B timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py tests/test_kmeans.py \
  > gpurun_out/r4j_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4j_tests.log; exit 1; }
tail -1 gpurun_out/r4j_tests.log
timeout -k 10 200 python -u tools/als_dense_phases.py --gl 1 > gpurun_out/r4j_phases_gl.json 2> gpurun_out/r4j_phases.err \
  || { echo "phases failed"; tail -20 gpurun_out/r4j_phases.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4j_phases_gl.json
for v in mfma_blk mfma_gl mfma_blk mfma_gl; do
  O3S_ALS_DENSE=$v timeout -k 10 200 python -u tools/bench_als.py --rank-of 8 --users 50000000 --items 5000000 \
    --ratings 1000000000 --iters 2 > gpurun_out/r4j_als_$v.json 2> gpurun_out/r4j_als_$v.err \
    || { echo "bench_als $v failed"; tail -20 gpurun_out/r4j_als_$v.err; exit 1; }
  echo "$v $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4j_als_$v.json').read().strip().splitlines()[-1]); print(d['value'], d.get('phases_s'))")"
done
for c in rows sums rows sums; do
  timeout -k 10 300 python -u tools/bench_kmeans.py --cost $c > gpurun_out/r4j_km_$c.json 2> gpurun_out/r4j_km_$c.err \
    || { echo "bench_kmeans $c failed"; tail -20 gpurun_out/r4j_km_$c.err; exit 1; }
  grep -v amdgpu.ids gpurun_out/r4j_km_$c.json
done
# GBT histogram after the round-3 conflict fix and the round-4 load ordering: kernel stats
# + PMC passes (kernel trace only), then the histogram micro-benchmark
timeout -k 10 900 bash tools/pmc_gbt_hist.sh || { echo "gbt pmc failed"; tail -5 gpurun_out/pmc_gbt/*.log; exit 1; }
cat gpurun_out/pmc_gbt/summary.txt
timeout -k 10 200 python -u tools/bench_hist.py > gpurun_out/r4j_hist.json 2>/dev/null || { echo "bench_hist failed"; exit 1; }
cat gpurun_out/r4j_hist.json
