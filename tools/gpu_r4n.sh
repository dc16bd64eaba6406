#!/bin/bash
# GBT full config: cold vs warm fit in one process (driver VRAM clearing on fresh hipMalloc).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 1 2; do
  timeout -k 10 300 python -u tools/bench_configs.py --config gbt --trees 5 --repeat 2 --out gpurun_out/r4n_gbt_rep$k.json > gpurun_out/r4n_gbt_rep$k.log 2>&1 \
    || { echo "gbt $k failed"; tail -20 gpurun_out/r4n_gbt_rep$k.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r4n_gbt_rep$k.json')); print(d['value'], d['fit_seconds_each'], d['alloc'], d['train_loss'])"
done
