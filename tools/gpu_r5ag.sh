#!/bin/bash
# Round 5: rehearsal of bench.py's multi-rank path on ONE GPU (2 and 4 ranks sharing
# cuda:0, gradient all-reduce over gloo) with a small row count -- the real SPMD code path
# with the real kernels; not a scaling measurement.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2 4; do
  O3S_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus $n --rows 40000000 --steps 5 --warmup 1 \
      --resident-fraction 0.1 > gpurun_out/r5ag_bench_n$n.json 2> gpurun_out/r5ag_bench_n$n.err \
    || { echo "bench n=$n failed"; tail -20 gpurun_out/r5ag_bench_n$n.err; exit 1; }
  tail -1 gpurun_out/r5ag_bench_n$n.json | cut -c1-400
done
