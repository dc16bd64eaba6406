#!/bin/bash
# Round 5: dense ALS kernel with DMA'd rating indices -- numerics, then phase clocks.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_als.py -m gpu \
  > gpurun_out/r5t_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r5t_tests.log; exit 1; }
tail -3 gpurun_out/r5t_tests.log
timeout -k 10 300 python -u tools/als_dense_phases.py > gpurun_out/r5t_phases.json 2> gpurun_out/r5t_phases.err \
  || { echo "phases failed"; tail -20 gpurun_out/r5t_phases.err; exit 1; }
cat gpurun_out/r5t_phases.json
