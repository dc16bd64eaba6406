#!/bin/bash
# r6: hist micro-benchmark + tree/kmeans tests + GBT full + KMeans blobs/uniform.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
bash tools/gpu_steps.sh \
  hist 200 python -u tools/bench_hist.py -- \
  km_tests 300 python -u -m pytest tests/test_kmeans.py tests/test_trees.py -m gpu -x -q --timeout 200 --timeout-method thread -- \
  gbt_full 300 python -u tools/bench_configs.py --config gbt --repeat 2 --out gpurun_out/gbt_full_r6.json -- \
  km_blobs 300 python -u tools/bench_kmeans_fit.py --repeat 2 --iters 10 -- \
  km_uniform 300 python -u tools/bench_kmeans_fit.py --repeat 2 --iters 10 --data uniform
