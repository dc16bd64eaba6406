#!/bin/bash
# Kernel-time breakdown of the GBT benchmark (rocprofv3 kernel trace only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_gbt
timeout -k 10 200 python3 tools/bench_gbt.py --trees 3 > gpurun_out/prof_gbt/bench.json 2>/dev/null \
&& (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_gbt/trace" \
    -o run -- python3 "$R/tools/bench_gbt.py" --trees 3) > gpurun_out/prof_gbt/prof.log 2>&1
