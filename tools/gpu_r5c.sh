#!/bin/bash
# dense wave kernel diagnostic: which tile / phase goes wrong at R >= 64
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug_dense_wave.py > gpurun_out/r5c_dbg.log 2>&1 || { echo "dbg failed"; tail -30 gpurun_out/r5c_dbg.log; exit 1; }
cat gpurun_out/r5c_dbg.log
