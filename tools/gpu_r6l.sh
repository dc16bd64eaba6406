#!/bin/bash
# r6: histogram LDS-DMA row stage -- A/B micro-benchmark, tree tests, GBT full config.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
bash tools/gpu_steps.sh \
  tree_tests 300 python -u -m pytest tests/test_trees.py -m gpu -x -q --timeout 200 --timeout-method thread -- \
  hist_dma 200 python -u tools/bench_hist.py -- \
  hist_gather 200 env O3S_HIST_DMA=0 python -u tools/bench_hist.py -- \
  gbt_full 300 python -u tools/bench_configs.py --config gbt --repeat 2 --out gpurun_out/gbt_full_r6.json -- \
  gbt_full_traced 300 python -u tools/bench_configs.py --config gbt --repeat 2 --trace --out gpurun_out/gbt_full_traced_r6.json
