#!/bin/bash
# Round 5: ALS full config (untraced, then kernel stats) on the final dense kernel + phases.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R="$PWD"
mkdir -p gpurun_out
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/r5aa_cfg_als.json > gpurun_out/r5aa_cfg_als.log 2>&1 \
  || { echo "als cfg failed"; tail -30 gpurun_out/r5aa_cfg_als.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5aa_cfg_als.json')); print('als', d['value'], d['fit_seconds'], d['iter_seconds'], d.get('session_warmup_s_untimed'))"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r5aa_als_stats" -o run -- \
   python3 "$R/tools/bench_configs.py" --config als --iters 3 --out "$R/gpurun_out/r5aa_cfg_als_prof.json") > gpurun_out/r5aa_als_stats.log 2>&1 \
  || { echo "als stats failed"; tail -20 gpurun_out/r5aa_als_stats.log; exit 1; }
grep -E "als_dense|als_wood" gpurun_out/r5aa_als_stats/run_kernel_stats.csv | cut -d, -f1-4 | sed 's/(.*)"/"/'
timeout -k 10 300 python -u tools/als_dense_phases.py > gpurun_out/r5aa_phases.json 2> gpurun_out/r5aa_phases.err \
  || { echo "phases failed"; tail -20 gpurun_out/r5aa_phases.err; exit 1; }
cat gpurun_out/r5aa_phases.json
