#!/bin/bash
# GBT histogram per-row rework (scalar row address, packed (w, w*y) LDS pairs, per-chunk
# vectorised weights) and the lean 3-blocks-per-CU KMeans screen: tests, then A/B timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_trees.py tests/test_kmeans.py tests/test_als.py \
  > gpurun_out/r4k_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4k_tests.log; exit 1; }
tail -1 gpurun_out/r4k_tests.log
for k in 1 2; do
  timeout -k 10 200 python -u tools/bench_gbt.py --trees 3 > gpurun_out/r4k_gbt_$k.json 2> gpurun_out/r4k_gbt_$k.err \
    || { echo "bench_gbt failed"; tail -20 gpurun_out/r4k_gbt_$k.err; exit 1; }
  echo "gbt $k $(python3 -c "import json; d=json.loads(open('gpurun_out/r4k_gbt_$k.json').read().strip().splitlines()[-1]); print(d['value'], d['loss'][-1])")"
done
timeout -k 10 200 python -u tools/bench_hist.py > gpurun_out/r4k_hist.json 2>/dev/null || { echo "bench_hist failed"; exit 1; }
cat gpurun_out/r4k_hist.json
for o in 2 3 2 3; do
  O3S_KM_SCREEN_OCC=$o timeout -k 10 300 python -u tools/bench_kmeans.py --cost sums > gpurun_out/r4k_km_$o.json 2> gpurun_out/r4k_km_$o.err \
    || { echo "bench_kmeans occ $o failed"; tail -20 gpurun_out/r4k_km_$o.err; exit 1; }
  echo "occ $o $(python3 -c "import json; d=json.loads(open('gpurun_out/r4k_km_$o.json').read().strip().splitlines()[-1]); print(round(d['ms_per_iter'],2), round(d['assign_ms'],2), d['cost'])")"
done
timeout -k 10 200 python -u tools/als_wood_phases.py > gpurun_out/r4k_wood_phases.json 2> gpurun_out/r4k_wood.err \
  || { echo "wood phases failed"; tail -20 gpurun_out/r4k_wood.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4k_wood_phases.json
