#!/bin/bash
# Round 5: the one-wave-per-row dense ALS kernel (numerics, A/B vs mfma_gl, full config)
# + the new multi-rank exact-ALS rehearsal and ADVICE regressions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 400 $T tests/test_als.py -k "dense or exact" > gpurun_out/r5b_als_tests.log 2>&1 \
  || { echo "als tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r5b_als_tests.log | head -20; tail -30 gpurun_out/r5b_als_tests.log; exit 1; }
tail -1 gpurun_out/r5b_als_tests.log
for K in wave mfma_gl; do
  O3S_ALS_DENSE=$K timeout -k 10 300 python -u tools/prof_als_exact.py --users 1000 --items 625000 --other 1000000 \
    --other-item 6250000 --reps 3 > gpurun_out/r5b_ab_$K.log 2>&1 || { echo "ab $K failed"; tail -20 gpurun_out/r5b_ab_$K.log; exit 1; }
  echo "$K: $(grep '^item' gpurun_out/r5b_ab_$K.log)"
done
timeout -k 10 500 $T tests/test_distributed_gpu.py tests/test_kmeans.py tests/test_spill.py > gpurun_out/r5b_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r5b_tests.log | head -20; tail -30 gpurun_out/r5b_tests.log; exit 1; }
tail -1 gpurun_out/r5b_tests.log
O3S_ALS_DENSE=wave timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/r5b_cfg_als.json > gpurun_out/r5b_cfg_als.log 2>&1 \
  || { echo "als cfg failed"; tail -30 gpurun_out/r5b_cfg_als.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5b_cfg_als.json')); print('full config', d['value'], d['fit_seconds'], d['iter_seconds'])"
