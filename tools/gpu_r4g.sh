#!/bin/bash
# ALS dense-kernel phase breakdown (diagnostic TIM build), then batch F.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/als_dense_phases.py > gpurun_out/r4g_phases.json 2> gpurun_out/r4g_phases.err \
  || { echo "phases failed"; tail -20 gpurun_out/r4g_phases.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r4g_phases.json
bash tools/gpu_r4f.sh
timeout -k 10 300 python -u tools/prof_fit_host.py > gpurun_out/r4g_prof_fit.json 2> gpurun_out/r4g_prof_fit.err || { echo 'prof fit failed'; tail -20 gpurun_out/r4g_prof_fit.err; exit 1; }
cat gpurun_out/r4g_prof_fit.json
