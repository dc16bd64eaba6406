#!/bin/bash
# Round 5 final: full GPU suite + smoke + 1-GPU bench (twice) on the final tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5final_gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; grep -E "FAILED|^E |Error" gpurun_out/r5final_gpu_tests.log | head -30; tail -5 gpurun_out/r5final_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r5final_gpu_tests.log
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5final_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r5final_smoke.log; exit 1; }
tail -1 gpurun_out/r5final_smoke.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > gpurun_out/r5final_bench_$i.json 2> gpurun_out/r5final_bench.err || { echo "bench failed"; tail -20 gpurun_out/r5final_bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5final_bench_$i.json')); print('bench', d['value']/1e9, d['ms_per_step'], d['hbm_only_rows_per_s']/1e9)"
done
