#!/bin/bash
# Round 5: k-means++ as two launches per step over the whole GPU (parity tests, init phases).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_kmeans.py > gpurun_out/r5p_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r5p_tests.log | head -30; tail -3 gpurun_out/r5p_tests.log; exit 1; }
tail -1 gpurun_out/r5p_tests.log
timeout -k 10 300 python -u tools/bench_kmeans_fit.py --iters 10 --repeat 2 > gpurun_out/r5p_kmeans_blobs.json 2> gpurun_out/r5p_kmeans_blobs.err \
  || { echo "kmeans blobs failed"; tail -20 gpurun_out/r5p_kmeans_blobs.err; exit 1; }
cut -c1-700 gpurun_out/r5p_kmeans_blobs.json
timeout -k 10 300 python -u tools/bench_kmeans_fit.py --iters 10 --repeat 2 --data uniform > gpurun_out/r5p_kmeans_uniform.json 2> gpurun_out/r5p_kmeans_uniform.err \
  || { echo "kmeans uniform failed"; tail -20 gpurun_out/r5p_kmeans_uniform.err; exit 1; }
cut -c1-700 gpurun_out/r5p_kmeans_uniform.json
