#!/bin/bash
# Round 5: k-means++ on fp32-rounded candidates, out-of-core staging, ALS in the moving eigenbasis.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 400 $T tests/test_kmeans.py tests/test_spill.py tests/test_feature.py > gpurun_out/r5i_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r5i_tests.log | head -30; tail -3 gpurun_out/r5i_tests.log; exit 1; }
tail -1 gpurun_out/r5i_tests.log
timeout -k 10 300 python -u tools/bench_kmeans_fit.py --iters 10 --repeat 2 > gpurun_out/r5i_kmeans_blobs.json 2> gpurun_out/r5i_kmeans_blobs.err \
  || { echo "kmeans blobs failed"; tail -20 gpurun_out/r5i_kmeans_blobs.err; exit 1; }
cut -c1-700 gpurun_out/r5i_kmeans_blobs.json
timeout -k 10 300 python -u tools/bench_kmeans_fit.py --iters 10 --repeat 2 --data uniform > gpurun_out/r5i_kmeans_uniform.json 2> gpurun_out/r5i_kmeans_uniform.err \
  || { echo "kmeans uniform failed"; tail -20 gpurun_out/r5i_kmeans_uniform.err; exit 1; }
cut -c1-700 gpurun_out/r5i_kmeans_uniform.json
timeout -k 10 300 python -u tools/bench_ooc.py > gpurun_out/r5i_ooc.json 2> gpurun_out/r5i_ooc.err || { echo "ooc failed"; tail -20 gpurun_out/r5i_ooc.err; exit 1; }
cat gpurun_out/r5i_ooc.json
timeout -k 10 500 $T tests/test_als.py tests/test_distributed_gpu.py tests/test_pool_models_recovery.py > gpurun_out/r5j_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r5j_tests.log | head -30; tail -3 gpurun_out/r5j_tests.log; exit 1; }
tail -1 gpurun_out/r5j_tests.log
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/r5j_cfg_als.json > gpurun_out/r5j_cfg_als.log 2>&1 \
  || { echo "als cfg failed"; tail -30 gpurun_out/r5j_cfg_als.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5j_cfg_als.json')); print('full config', d['value'], d['fit_seconds'], d['iter_seconds'])"
timeout -k 10 400 $T tests/test_trees.py tests/test_gpu_estimators.py > gpurun_out/r5l_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r5l_tests.log | head -30; tail -3 gpurun_out/r5l_tests.log; exit 1; }
tail -1 gpurun_out/r5l_tests.log
timeout -k 10 400 python -u tools/bench_configs.py --config gbt --repeat 2 --out gpurun_out/r5l_cfg_gbt.json > gpurun_out/r5l_cfg_gbt.log 2>&1 \
  || { echo "gbt cfg failed"; tail -20 gpurun_out/r5l_cfg_gbt.log; exit 1; }
cut -c1-900 gpurun_out/r5l_cfg_gbt.json
timeout -k 10 400 python -u tools/bench_configs.py --config gbt --repeat 2 --trace --out gpurun_out/r5l_cfg_gbt_traced.json > gpurun_out/r5l_cfg_gbt_traced.log 2>&1 \
  || { echo "gbt traced failed"; tail -20 gpurun_out/r5l_cfg_gbt_traced.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5l_cfg_gbt_traced.json')); print(d['value'], d.get('fit_seconds_each'), json.dumps(d.get('phases_s'))[:900])"
