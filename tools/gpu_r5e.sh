#!/bin/bash
# Round 5: full GPU suite + smoke on the single dense ALS kernel, then profiles: ALS full
# config kernel stats + PMC of the wave kernel, KMeans fit cold/warm (blobs, uniform), GBT
# cold/warm + peak, out-of-core ingest rate, HashingTF kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R="$PWD"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5e_gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; grep -E "FAILED|^E |Error" gpurun_out/r5e_gpu_tests.log | head -30; tail -5 gpurun_out/r5e_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r5e_gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5e_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r5e_smoke.log; exit 1; }
tail -1 gpurun_out/r5e_smoke.log
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r5e_als_stats" -o run -- \
   python3 "$R/tools/bench_configs.py" --config als --iters 3 --out "$R/gpurun_out/r5e_cfg_als_traced.json") > gpurun_out/r5e_als_stats.log 2>&1 \
  || { echo "als stats failed"; tail -20 gpurun_out/r5e_als_stats.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5e_cfg_als_traced.json')); print('als traced', d['value'], d['iter_seconds'])"
timeout -k 10 300 python -u tools/bench_kmeans_fit.py --iters 10 --repeat 2 > gpurun_out/r5e_kmeans_blobs.json 2> gpurun_out/r5e_kmeans_blobs.err \
  || { echo "kmeans blobs failed"; tail -20 gpurun_out/r5e_kmeans_blobs.err; exit 1; }
cut -c1-700 gpurun_out/r5e_kmeans_blobs.json
timeout -k 10 300 python -u tools/bench_kmeans_fit.py --iters 10 --repeat 2 --data uniform > gpurun_out/r5e_kmeans_uniform.json 2> gpurun_out/r5e_kmeans_uniform.err \
  || { echo "kmeans uniform failed"; tail -20 gpurun_out/r5e_kmeans_uniform.err; exit 1; }
cut -c1-700 gpurun_out/r5e_kmeans_uniform.json
timeout -k 10 400 python -u tools/bench_configs.py --config gbt --repeat 2 --out gpurun_out/r5e_cfg_gbt.json > gpurun_out/r5e_cfg_gbt.log 2>&1 \
  || { echo "gbt cfg failed"; tail -20 gpurun_out/r5e_cfg_gbt.log; exit 1; }
cut -c1-900 gpurun_out/r5e_cfg_gbt.json
timeout -k 10 300 python -u tools/bench_ooc.py > gpurun_out/r5e_ooc.json 2> gpurun_out/r5e_ooc.err || { echo "ooc failed"; tail -20 gpurun_out/r5e_ooc.err; exit 1; }
cat gpurun_out/r5e_ooc.json
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r5e_text_stats" -o run -- \
   python3 "$R/tools/bench_text.py") > gpurun_out/r5e_text_stats.log 2>&1 || { echo "text stats failed"; tail -20 gpurun_out/r5e_text_stats.log; exit 1; }
echo "text stats ok"
bash tools/pmc_als_exact.sh > gpurun_out/r5e_pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/r5e_pmc.log; exit 1; }
cat gpurun_out/pmc_als/summary_dense.txt | head -40
