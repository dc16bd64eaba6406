#!/bin/bash
# DRAM bytes per dispatch of the streaming kernels (GLM gradient pass, VectorAssembler,
# KMeans assign/update), counted at the TCC->EA interface.  On gfx950 the derived
# FETCH_SIZE counts a 128-byte request as 64 bytes, so the pass reads the per-sector
# counter (TCC_EA0_RDREQ_DRAM_32B: a 128-byte request counts 4) next to the 128-byte
# request count.  One counter pass per program, each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
O=gpurun_out/pmc_bytes
mkdir -p $O
export TMPDIR=/tmp
C="TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE"
run() {  # name, program args...
  local n=$1; shift
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$R/$O/$n" -o run -- python3 "$@") \
    > $O/$n.log 2>&1
}
run glm "$R/tools/bench_glm_kernel.py" --iters 2 \
&& run assemble "$R/tools/bench_assemble.py" --reps 2 \
&& run kmeans "$R/tools/bench_kmeans.py" --rows 20000000 --iters 2
rc=$?
python3 tools/pmc_bytes.py $O > $O/summary.txt
exit $rc
