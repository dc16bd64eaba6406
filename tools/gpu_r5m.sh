#!/bin/bash
# Round 5: full GPU suite + smoke after the kernel changes; KMeans init with Spark's
# single-draw k-means++; out-of-core ingest host split; GBT per-fit phases (cold vs warm).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5m_gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; grep -E "FAILED|^E " gpurun_out/r5m_gpu_tests.log | head -30; tail -5 gpurun_out/r5m_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r5m_gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5m_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r5m_smoke.log; exit 1; }
tail -1 gpurun_out/r5m_smoke.log
timeout -k 10 300 python -u tools/bench_kmeans_fit.py --iters 10 --repeat 2 > gpurun_out/r5m_kmeans_blobs.json 2> gpurun_out/r5m_kmeans_blobs.err \
  || { echo "kmeans blobs failed"; tail -20 gpurun_out/r5m_kmeans_blobs.err; exit 1; }
cut -c1-700 gpurun_out/r5m_kmeans_blobs.json
timeout -k 10 300 python -u tools/bench_kmeans_fit.py --iters 10 --repeat 2 --data uniform > gpurun_out/r5m_kmeans_uniform.json 2> gpurun_out/r5m_kmeans_uniform.err \
  || { echo "kmeans uniform failed"; tail -20 gpurun_out/r5m_kmeans_uniform.err; exit 1; }
cut -c1-700 gpurun_out/r5m_kmeans_uniform.json
timeout -k 10 300 python -u tools/bench_ooc.py > gpurun_out/r5m_ooc.json 2> gpurun_out/r5m_ooc.err || { echo "ooc failed"; tail -20 gpurun_out/r5m_ooc.err; exit 1; }
cat gpurun_out/r5m_ooc.json
timeout -k 10 400 python -u tools/bench_configs.py --config gbt --repeat 2 --trace --out gpurun_out/r5m_cfg_gbt_traced.json > gpurun_out/r5m_cfg_gbt_traced.log 2>&1 \
  || { echo "gbt traced failed"; tail -20 gpurun_out/r5m_cfg_gbt_traced.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5m_cfg_gbt_traced.json')); print(d['fit_seconds_each'], json.dumps(d.get('phases_each_fit_s'))[:1500])"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r5m_bench.json 2> gpurun_out/r5m_bench.err || { echo "bench failed"; tail -20 gpurun_out/r5m_bench.err; exit 1; }
cat gpurun_out/r5m_bench.json
