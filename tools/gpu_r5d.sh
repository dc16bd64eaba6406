#!/bin/bash
# Round 5: wave dense ALS kernel (numerics after the lane-sync fix, A/B, full config),
# HashingTF per-document kernels, out-of-core ingest, multi-rank exact-ALS rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 300 python -u tools/debug_dense_wave.py > gpurun_out/r5d_dbg.log 2>&1 || { echo "dbg failed"; tail -30 gpurun_out/r5d_dbg.log; exit 1; }
grep -E "^(64|128) " gpurun_out/r5d_dbg.log | cut -c1-60
timeout -k 10 400 $T tests/test_als.py -k "dense or exact" > gpurun_out/r5d_als_tests.log 2>&1 \
  || { echo "als tests failed"; grep -E "FAILED|^E " gpurun_out/r5d_als_tests.log | head -20; exit 1; }
tail -1 gpurun_out/r5d_als_tests.log
for K in wave mfma_gl; do
  O3S_ALS_DENSE=$K timeout -k 10 300 python -u tools/prof_als_exact.py --users 1000 --items 625000 --other 1000000 \
    --other-item 6250000 --reps 3 > gpurun_out/r5d_ab_$K.log 2>&1 || { echo "ab $K failed"; tail -20 gpurun_out/r5d_ab_$K.log; exit 1; }
  echo "$K: $(grep '^item' gpurun_out/r5d_ab_$K.log | cut -c1-220)"
done
timeout -k 10 500 $T tests/test_feature.py -k "hashingtf or tokenizer" tests/test_spill.py tests/test_distributed_gpu.py tests/test_kmeans.py \
  > gpurun_out/r5d_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r5d_tests.log | head -20; tail -5 gpurun_out/r5d_tests.log; exit 1; }
tail -1 gpurun_out/r5d_tests.log
O3S_ALS_DENSE=wave timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/r5d_cfg_als.json > gpurun_out/r5d_cfg_als.log 2>&1 \
  || { echo "als cfg failed"; tail -30 gpurun_out/r5d_cfg_als.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5d_cfg_als.json')); print('full config', d['value'], d['fit_seconds'], d['iter_seconds'])"
timeout -k 10 300 python -u tools/bench_text.py > gpurun_out/r5d_text.json 2> gpurun_out/r5d_text.err || { echo "text bench failed"; tail -20 gpurun_out/r5d_text.err; exit 1; }
cat gpurun_out/r5d_text.json
timeout -k 10 300 $T tests/test_kmeans.py -k kmeanspp > gpurun_out/r5d_kpp.log 2>&1 || { echo "kmeanspp test failed"; grep -E "FAILED|^E " gpurun_out/r5d_kpp.log | head; exit 1; }
tail -1 gpurun_out/r5d_kpp.log
timeout -k 10 300 python -u tools/bench_kmeans_fit.py --iters 10 > gpurun_out/r5d_kmeans_fit.json 2> gpurun_out/r5d_kmeans_fit.err || { echo "kmeans fit failed"; tail -20 gpurun_out/r5d_kmeans_fit.err; exit 1; }
cat gpurun_out/r5d_kmeans_fit.json
