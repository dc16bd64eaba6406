#!/bin/bash
# r6: KMeans uniform kernel stats + kmeans tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
R=$GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
  km_tests 300 python -u -m pytest tests/test_kmeans.py -m gpu -x -q --timeout 200 --timeout-method thread -- \
  prof_km_uniform 300 bash tools/prof_step.sh prof_km_uniform_r6 python3 $R/tools/bench_kmeans_fit.py --repeat 1 --iters 10 --data uniform
