#!/bin/bash
# Round 5: KMeans uniform data, Lloyd with and without the pair screen (PAIR_FROM A/B).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_kmeans_fit.py --iters 10 --repeat 2 --data uniform > gpurun_out/r5af_uniform_plain.json 2> gpurun_out/r5af.err \
  || { echo "plain failed"; tail -20 gpurun_out/r5af.err; exit 1; }
tail -1 gpurun_out/r5af_uniform_plain.json | cut -c1-600
timeout -k 10 300 python -u tools/bench_kmeans_fit.py --iters 10 --repeat 2 --data uniform --pair-from 0.05 > gpurun_out/r5af_uniform_pair.json 2> gpurun_out/r5af.err \
  || { echo "pair failed"; tail -20 gpurun_out/r5af.err; exit 1; }
tail -1 gpurun_out/r5af_uniform_pair.json | cut -c1-600
