#!/bin/bash
# r6: is the histogram kernel bound by the texture addresser (per-row byte gathers)?
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
R=$GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
  pmc_hist_ta 120 bash tools/pmc_step.sh pmc_hist_ta_r6 "tree_hist" "TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE GRBM_COUNT" python3 $R/tools/bench_hist.py 20000000 -- \
  pmc_hist_sq 120 bash tools/pmc_step.sh pmc_hist_sq_r6 "tree_hist" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" python3 $R/tools/bench_hist.py 20000000
