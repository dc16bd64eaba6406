#!/bin/bash
# Round 5: GBT cold vs warm fit with and without a tiny prewarm fit (is the cold cost first-use?).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_configs.py --config gbt --repeat 2 --trace --out gpurun_out/r5y_gbt_plain.json > gpurun_out/r5y_gbt_plain.log 2>&1 \
  || { echo "gbt failed"; tail -20 gpurun_out/r5y_gbt_plain.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5y_gbt_plain.json')); print('plain', d['fit_seconds_each'], d['phases_each_fit_s'])"
timeout -k 10 400 python -u tools/bench_configs.py --config gbt --repeat 2 --trace --prewarm --out gpurun_out/r5y_gbt_prewarm.json > gpurun_out/r5y_gbt_prewarm.log 2>&1 \
  || { echo "gbt prewarm failed"; tail -20 gpurun_out/r5y_gbt_prewarm.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5y_gbt_prewarm.json')); print('prewarm', d['fit_seconds_each'], d['phases_each_fit_s'])"
grep prewarm gpurun_out/r5y_gbt_prewarm.log
