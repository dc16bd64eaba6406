#!/bin/bash
# r6: GBT fused epilogue -- tree GPU tests, then the full GBT config (untraced + traced).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
bash tools/gpu_steps.sh \
  tree_tests 300 python -u -m pytest tests/test_trees.py -m gpu -x -q --timeout 200 --timeout-method thread -- \
  gbt_full 300 python -u tools/bench_configs.py --config gbt --repeat 2 --out gpurun_out/gbt_full_r6.json -- \
  gbt_full_traced 300 python -u tools/bench_configs.py --config gbt --repeat 2 --trace --out gpurun_out/gbt_full_traced_r6.json
