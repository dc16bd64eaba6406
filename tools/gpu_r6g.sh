#!/bin/bash
# r6: kmeans + tree GPU tests, GBT kernel stats, KMeans Lloyd timing (clustered + uniform).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
R=$GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
  hist_pairs 200 python -u tools/bench_hist.py -- \
  hist_nopairs 200 env O3S_HIST_PAIRS=0 python -u tools/bench_hist.py -- \
  km_tests 300 python -u -m pytest tests/test_kmeans.py tests/test_trees.py -m gpu -x -q --timeout 200 --timeout-method thread -- \
  prof_gbt 300 bash tools/prof_step.sh prof_gbt_r6 python3 $R/tools/bench_configs.py --config gbt --rows 100000000 --trees 3 --repeat 1 -- \
  km_blobs 300 python -u tools/bench_kmeans_fit.py --repeat 2 --iters 10 -- \
  km_blobs_full 300 python -u tools/bench_kmeans_fit.py --repeat 2 --iters 10 --no-hamerly -- \
  km_uniform 300 python -u tools/bench_kmeans_fit.py --repeat 2 --iters 10 --data uniform
