#!/bin/bash
# Round 5, first GPU check: the new multi-rank exact-ALS rehearsal + ADVICE regressions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py tests/test_kmeans.py tests/test_spill.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r5a_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5a_tests.log; exit 1; }
tail -3 gpurun_out/r5a_tests.log
