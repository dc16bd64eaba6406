#!/bin/bash
# KMeans screen PMC: the no-distance pre-split build of the Lloyd iterations vs the
# per-row-distance build (20M x 128, k = 1024, blobs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
SCR_ARGS="--nodist" timeout -k 10 400 bash tools/pmc_kmeans_screen.sh || { echo "pmc nodist failed"; tail -5 gpurun_out/pmc_scr/*.log; exit 1; }
mv gpurun_out/pmc_scr gpurun_out/pmc_scr_nodist
cat gpurun_out/pmc_scr_nodist/summary.txt
timeout -k 10 400 bash tools/pmc_kmeans_screen.sh || { echo "pmc dist failed"; tail -5 gpurun_out/pmc_scr/*.log; exit 1; }
cat gpurun_out/pmc_scr/summary.txt
grep -h "done" gpurun_out/pmc_scr_nodist/p1.log gpurun_out/pmc_scr/p1.log
