#!/bin/bash
# Round 5: Woodbury kernel phase clocks per launch width (16: 1..16 ratings, 24: 17..24, 32: 25..32).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for kn in 16 24 32; do
  timeout -k 10 200 python -u tools/als_wood_phases.py --kn $kn > gpurun_out/r5ab_wood_$kn.json 2> gpurun_out/r5ab_wood.err \
    || { echo "wood $kn failed"; tail -20 gpurun_out/r5ab_wood.err; exit 1; }
  cat gpurun_out/r5ab_wood_$kn.json
done
