#!/bin/bash
# Round 5: ALS full config under rocprofv3 kernel stats (dense kernel with DMA'd indices /
# metadata and pk_fma diagonal) + PMC of the exact ALS kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R="$PWD"
mkdir -p gpurun_out
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r5w_als_stats" -o run -- \
   python3 "$R/tools/bench_configs.py" --config als --iters 3 --out "$R/gpurun_out/r5w_cfg_als_traced.json") > gpurun_out/r5w_als_stats.log 2>&1 \
  || { echo "als stats failed"; tail -20 gpurun_out/r5w_als_stats.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5w_cfg_als_traced.json')); print('als traced', d['value'], d['iter_seconds'])"
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/r5w_cfg_als.json > gpurun_out/r5w_cfg_als.log 2>&1 \
  || { echo "als cfg failed"; tail -30 gpurun_out/r5w_cfg_als.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5w_cfg_als.json')); print('als', d['value'], d['fit_seconds'], d['iter_seconds'])"
bash tools/pmc_als_exact.sh > gpurun_out/r5w_pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/r5w_pmc.log; exit 1; }
head -40 gpurun_out/pmc_als/summary_dense.txt
timeout -k 10 300 python -u tools/als_wood_phases.py > gpurun_out/r5w_wood_phases.json 2> gpurun_out/r5w_wood_phases.err \
  || { echo "wood phases failed"; tail -20 gpurun_out/r5w_wood_phases.err; exit 1; }
cat gpurun_out/r5w_wood_phases.json
