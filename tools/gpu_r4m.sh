#!/bin/bash
# Round-4 batch M: the whole GPU suite, smoke(), the N=1 headline bench + its kernel stats,
# the full ALS / GBT configs at N=1, the KMeans Lloyd bench, the fit-level KMeans bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r4m_gputests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/r4m_gputests.log | head -20; tail -30 gpurun_out/r4m_gputests.log; exit 1; }
tail -1 gpurun_out/r4m_gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4m_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4m_smoke.log; exit 1; }
tail -1 gpurun_out/r4m_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r4m_bench.json 2> gpurun_out/r4m_bench.err || { echo "bench failed"; tail -20 gpurun_out/r4m_bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4m_bench.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r4m_prof_bench" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2) \
  > gpurun_out/r4m_prof_bench.log 2>&1 || { echo "bench profile failed"; tail -20 gpurun_out/r4m_prof_bench.log; exit 1; }
head -5 gpurun_out/r4m_prof_bench/run_kernel_stats.csv | cut -c1-150
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/r4m_cfg_als.json > gpurun_out/r4m_cfg_als.log 2>&1 || { echo "als cfg failed"; tail -30 gpurun_out/r4m_cfg_als.log; exit 1; }
cat gpurun_out/r4m_cfg_als.json
timeout -k 10 420 python -u tools/bench_configs.py --config gbt --trees 5 --out gpurun_out/r4m_cfg_gbt.json > gpurun_out/r4m_cfg_gbt.log 2>&1 || { echo "gbt cfg failed"; tail -30 gpurun_out/r4m_cfg_gbt.log; exit 1; }
cat gpurun_out/r4m_cfg_gbt.json
timeout -k 10 300 python -u tools/bench_kmeans.py > gpurun_out/r4m_km.json 2> gpurun_out/r4m_km.err || { echo "kmeans failed"; tail -20 gpurun_out/r4m_km.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4m_km.json
timeout -k 10 400 python -u tools/bench_kmeans_fit.py --iters 10 > gpurun_out/r4m_km_fit.json 2> gpurun_out/r4m_km_fit.err || { echo "kmeans fit failed"; tail -20 gpurun_out/r4m_km_fit.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4m_km_fit.json
