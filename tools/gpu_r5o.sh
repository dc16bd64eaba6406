#!/bin/bash
# Round 5: dense ALS explicit variant with the 4-step ring (numerics; item-side explicit vs
# implicit timing as a ring-depth probe); gather-table-size probe (implicit item side from
# a 1M- vs 6.25M- vs 25M-row table).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 400 $T tests/test_als.py -k "dense or exact" > gpurun_out/r5o_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r5o_tests.log | head -30; tail -3 gpurun_out/r5o_tests.log; exit 1; }
tail -1 gpurun_out/r5o_tests.log
for other in 1000000 6250000 25000000; do
  timeout -k 10 300 python -u tools/prof_als_exact.py --users 1000 --items 625000 --other 1000000 --other-item $other --reps 3 \
    > gpurun_out/r5o_imp_$other.log 2>&1 || { echo "imp $other failed"; tail -20 gpurun_out/r5o_imp_$other.log; exit 1; }
  echo "implicit other=$other: $(grep '^item' gpurun_out/r5o_imp_$other.log | cut -c1-200)"
done
timeout -k 10 300 python -u tools/prof_als_exact.py --users 1000 --items 625000 --other 1000000 --other-item 6250000 --reps 3 --explicit \
  > gpurun_out/r5o_exp.log 2>&1 || { echo "exp failed"; tail -20 gpurun_out/r5o_exp.log; exit 1; }
echo "explicit (4-step ring): $(grep '^item' gpurun_out/r5o_exp.log | cut -c1-200)"
timeout -k 10 300 $T tests/test_kmeans.py > gpurun_out/r5o_kmeans_tests.log 2>&1 \
  || { echo "kmeans tests failed"; grep -E "FAILED|^E " gpurun_out/r5o_kmeans_tests.log | head -20; exit 1; }
tail -1 gpurun_out/r5o_kmeans_tests.log
timeout -k 10 300 python -u tools/bench_kmeans_fit.py --iters 10 --repeat 2 > gpurun_out/r5o_kmeans_blobs.json 2> gpurun_out/r5o_kmeans_blobs.err \
  || { echo "kmeans blobs failed"; tail -20 gpurun_out/r5o_kmeans_blobs.err; exit 1; }
cut -c1-700 gpurun_out/r5o_kmeans_blobs.json
timeout -k 10 120 python -u tools/probe_kmeanspp.py > gpurun_out/r5o_kpp_probe.json 2>&1 || { echo 'kpp probe failed'; tail -20 gpurun_out/r5o_kpp_probe.json; exit 1; }
cat gpurun_out/r5o_kpp_probe.json
