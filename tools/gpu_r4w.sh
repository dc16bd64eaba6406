#!/bin/bash
# Round-4 end-state measurements: KMeans structureless data, GBT per-rank share, GBT full config.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_kmeans.py --data uniform > gpurun_out/r4w_km_uniform.json 2> gpurun_out/r4w_km_uniform.err || { echo "kmeans uniform failed"; tail -20 gpurun_out/r4w_km_uniform.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4w_km_uniform.json
for k in 1 2; do
  timeout -k 10 200 python -u tools/bench_gbt.py --trees 5 > gpurun_out/r4w_gbt_$k.json 2> gpurun_out/r4w_gbt_$k.err \
    || { echo "bench_gbt failed"; tail -20 gpurun_out/r4w_gbt_$k.err; exit 1; }
  echo "gbt $k $(python3 -c "import json; d=json.loads(open('gpurun_out/r4w_gbt_$k.json').read().strip().splitlines()[-1]); print(d['value'], d['loss'][-1])")"
done
timeout -k 10 400 python -u tools/bench_configs.py --config gbt --trees 5 --repeat 2 --out gpurun_out/r4w_cfg_gbt.json > gpurun_out/r4w_cfg_gbt.log 2>&1 || { echo "gbt cfg failed"; tail -30 gpurun_out/r4w_cfg_gbt.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4w_cfg_gbt.json')); print(d['value'], d['fit_seconds_each'], d['train_loss'])"
