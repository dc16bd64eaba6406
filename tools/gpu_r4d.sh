#!/bin/bash
# Round-4 GPU batch D: KMeans pre-split screen -- correctness, A/B at 100M x 128 k=1024, PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kmeans.py \
  > gpurun_out/r4d_km_tests.log 2>&1 || { echo "kmeans tests failed"; tail -40 gpurun_out/r4d_km_tests.log; exit 1; }
tail -2 gpurun_out/r4d_km_tests.log
for ps in off on off on; do
  timeout -k 10 300 python -u tools/bench_kmeans.py --mode auto --presplit $ps > gpurun_out/r4d_km_$ps.json 2> gpurun_out/r4d_km_$ps.err \
    || { echo "bench kmeans $ps failed"; tail -20 gpurun_out/r4d_km_$ps.err; exit 1; }
  echo "$ps $(tail -1 gpurun_out/r4d_km_$ps.json)"
done
SCR_ARGS="--rows 20000000" timeout -k 10 400 bash tools/pmc_kmeans_screen.sh || { echo "pmc kmeans failed"; exit 1; }
cat gpurun_out/pmc_scr/summary.txt
timeout -k 10 420 python -u tools/bench_pool_als.py > gpurun_out/r4d_pool_als.log 2>&1 || { echo "pool als failed"; tail -30 gpurun_out/r4d_pool_als.log; exit 1; }
tail -1 gpurun_out/r4d_pool_als.log
