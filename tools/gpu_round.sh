#!/bin/bash
# One GPU-box pass: gpu tests, smoke, 1-GPU bench, kernel-trace stats of the bench.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 \
&& timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
&& timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 \
&& if [ "${PROFILE:-1}" = 1 ]; then
     (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench" \
        -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2) > gpurun_out/prof_bench.log 2>&1
   fi
rc=$?
tail -3 gpurun_out/gpu_tests.log; tail -2 gpurun_out/smoke.log 2>/dev/null; tail -2 gpurun_out/bench.log 2>/dev/null
exit $rc
