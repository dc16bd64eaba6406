#!/bin/bash
# Round 5: Woodbury with symmetric multipliers -- ALS GPU tests, then phase clocks per width.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_als.py -m gpu \
  > gpurun_out/r5ad_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r5ad_tests.log; exit 1; }
tail -1 gpurun_out/r5ad_tests.log
for kn in 16 24 32; do
  timeout -k 10 200 python -u tools/als_wood_phases.py --kn $kn > gpurun_out/r5ad_wood_$kn.json 2> gpurun_out/r5ad_wood.err \
    || { echo "wood $kn failed"; tail -20 gpurun_out/r5ad_wood.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5ad_wood_$kn.json')); print($kn, round(d['production_ms'],3), d['cycles_per_row_mean'])"
done
