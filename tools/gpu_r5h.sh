#!/bin/bash
# Round 5: dense ALS Gram software-pipelined (fragments of step s+1 beside the MFMAs of
# step s, raw v_sqrt): numerics, item-side A/B vs r5f (31.2 ms), full config; k-means++
# register blocking (init phases); out-of-core ingest with pinned staging.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 500 $T tests/test_als.py tests/test_kmeans.py tests/test_spill.py > gpurun_out/r5h_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r5h_tests.log | head -30; tail -3 gpurun_out/r5h_tests.log; exit 1; }
tail -1 gpurun_out/r5h_tests.log
timeout -k 10 300 python -u tools/prof_als_exact.py --users 1000 --items 625000 --other 1000000 --other-item 6250000 --reps 3 \
  > gpurun_out/r5h_ab_item.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/r5h_ab_item.log; exit 1; }
echo "item: $(grep '^item' gpurun_out/r5h_ab_item.log | cut -c1-220)"
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/r5h_cfg_als.json > gpurun_out/r5h_cfg_als.log 2>&1 \
  || { echo "als cfg failed"; tail -30 gpurun_out/r5h_cfg_als.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5h_cfg_als.json')); print('full config', d['value'], d['fit_seconds'], d['iter_seconds'])"
timeout -k 10 300 python -u tools/bench_kmeans_fit.py --iters 10 --repeat 2 > gpurun_out/r5h_kmeans_blobs.json 2> gpurun_out/r5h_kmeans_blobs.err \
  || { echo "kmeans blobs failed"; tail -20 gpurun_out/r5h_kmeans_blobs.err; exit 1; }
cut -c1-700 gpurun_out/r5h_kmeans_blobs.json
timeout -k 10 300 python -u tools/bench_ooc.py > gpurun_out/r5h_ooc.json 2> gpurun_out/r5h_ooc.err || { echo "ooc failed"; tail -20 gpurun_out/r5h_ooc.err; exit 1; }
cat gpurun_out/r5h_ooc.json
