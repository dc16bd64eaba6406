#!/bin/bash
# r6: tree GPU tests + kernel stats of the GBT config (100M rows, 3 trees) + leaf-pass PMC.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
R=$GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
  tree_tests 300 python -u -m pytest tests/test_trees.py -m gpu -x -q --timeout 200 --timeout-method thread -- \
  prof_gbt 300 bash tools/prof_step.sh prof_gbt_r6 python3 $R/tools/bench_configs.py --config gbt --rows 100000000 --trees 3 --repeat 1 -- \
  pmc_leaf 120 bash tools/pmc_step.sh pmc_leaf_r6 "gbt_leaf|tree_hist" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" python3 $R/tools/bench_configs.py --config gbt --rows 20000000 --trees 2 --repeat 1
