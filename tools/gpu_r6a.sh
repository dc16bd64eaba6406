#!/bin/bash
# r6 first pass: GPU suite, smoke, bench, cold-start probes.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
P="python -u tools/probe_coldstart.py"
bash tools/gpu_steps.sh \
  gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -- \
  smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()" -- \
  bench 300 python -u bench.py -- \
  cold_none 120 $P --mode none -- \
  cold_preload 120 $P --mode preload -- \
  cold_family 120 $P --mode family -- \
  cold_fits 120 $P --mode fits -- \
  cold_deferred0 240 env HIP_ENABLE_DEFERRED_LOADING=0 $P --mode none -- \
  cold_glm_none 120 $P --mode none --family glm -- \
  cold_glm_preload 120 $P --mode preload --family glm -- \
  cold_glm_family 120 $P --mode family --family glm
