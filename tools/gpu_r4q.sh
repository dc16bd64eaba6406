#!/bin/bash
# Woodbury S build bf16x3 (opt-in) vs exact fp32: tests, kernel time, rank-of-8 iteration;
# then the KMeans screen PMC (no-distance vs per-row-distance builds).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
O3S_ALS_WOOD_S3=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py \
  > gpurun_out/r4q_tests_s3.log 2>&1 || { echo "s3 tests failed"; grep -E "assert|Error" gpurun_out/r4q_tests_s3.log | head -10; tail -5 gpurun_out/r4q_tests_s3.log; }
tail -1 gpurun_out/r4q_tests_s3.log
for s3 in 0 1 0 1; do
  timeout -k 10 200 python -u tools/als_wood_phases.py --s3 $s3 > gpurun_out/r4q_wood_$s3.json 2>/dev/null || { echo "wood $s3 failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r4q_wood_$s3.json').read().strip().splitlines()[-1]); print('s3', $s3, round(d['production_ms'],3))"
done
for s3 in 0 1; do
  O3S_ALS_WOOD_S3=$s3 timeout -k 10 200 python -u tools/bench_als.py --rank-of 8 --users 50000000 --items 5000000 \
    --ratings 1000000000 --iters 2 > gpurun_out/r4q_als_$s3.json 2> gpurun_out/r4q_als_$s3.err \
    || { echo "bench_als $s3 failed"; tail -20 gpurun_out/r4q_als_$s3.err; exit 1; }
  echo "als s3=$s3 $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4q_als_$s3.json').read().strip().splitlines()[-1]); print(d['value'])")"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_als.py -k dense_kernels \
  > gpurun_out/r4q_gd_tests.log 2>&1 || { echo "gd tests failed"; tail -30 gpurun_out/r4q_gd_tests.log; exit 1; }
tail -1 gpurun_out/r4q_gd_tests.log
timeout -k 10 200 python -u tools/als_dense_phases.py --gl 1 > gpurun_out/r4q_phases.json 2>/dev/null || { echo "phases failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/r4q_phases.json
for v in mfma_gl mfma_gd mfma_gl mfma_gd; do
  O3S_ALS_DENSE=$v timeout -k 10 200 python -u tools/bench_als.py --rank-of 8 --users 50000000 --items 5000000 \
    --ratings 1000000000 --iters 2 > gpurun_out/r4q_als_$v.json 2> gpurun_out/r4q_als_$v.err \
    || { echo "bench_als $v failed"; tail -20 gpurun_out/r4q_als_$v.err; exit 1; }
  echo "$v $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4q_als_$v.json').read().strip().splitlines()[-1]); print(d['value'])")"
done
timeout -k 10 900 bash tools/gpu_r4p.sh
# verification of the current defaults: the whole GPU suite, smoke(), the N=1 bench
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r4q_gputests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/r4q_gputests.log | head -20; tail -20 gpurun_out/r4q_gputests.log; exit 1; }
tail -1 gpurun_out/r4q_gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4q_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4q_smoke.log; exit 1; }
tail -1 gpurun_out/r4q_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r4q_bench.json 2> gpurun_out/r4q_bench.err || { echo "bench failed"; tail -20 gpurun_out/r4q_bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4q_bench.json
