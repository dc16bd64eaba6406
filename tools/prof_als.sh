#!/bin/bash
# Kernel-time breakdown of the ALS benchmark (rocprofv3 kernel trace only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_als
timeout -k 10 300 python3 tools/bench_als.py > gpurun_out/prof_als/bench.json 2>/dev/null \
&& (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_als/trace" \
    -o run -- python3 "$R/tools/bench_als.py") > gpurun_out/prof_als/prof.log 2>&1
