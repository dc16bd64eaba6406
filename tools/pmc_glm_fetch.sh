#!/bin/bash
# GLM gradient pass (125M x 256 bf16 resident + the lineage pass): HBM bytes fetched per
# dispatch (FETCH_SIZE, KiB) next to the kernel trace, to pin the bandwidth claim on a
# counter rather than on timing alone.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
mkdir -p gpurun_out/pmc_glm
export TMPDIR=/tmp
B="$R/tools/bench_glm_kernel.py --iters 2"
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pmc_glm/stats" \
    -o run -- python3 $B) > gpurun_out/pmc_glm/stats.log 2>&1 \
&& (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES \
    --output-format csv -d "$R/gpurun_out/pmc_glm/p1" -o run -- python3 $B) > gpurun_out/pmc_glm/p1.log 2>&1 \
&& (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/pmc_glm/p2" -o run -- python3 $B) > gpurun_out/pmc_glm/p2.log 2>&1
rc=$?
python3 tools/pmc_summary.py gpurun_out/pmc_glm glm_grad > gpurun_out/pmc_glm/summary.txt
exit $rc
