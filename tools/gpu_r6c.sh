#!/bin/bash
# r6: GPU suite with the background warm-up, then the cold-start protocol per mode.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
P="python -u tools/probe_coldstart.py"
bash tools/gpu_steps.sh \
  gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -- \
  smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()" -- \
  cold_auto_trees 200 $P --mode auto --rows 500000000 -- \
  cold_none_trees 200 $P --mode none --rows 500000000 -- \
  cold_auto_glm 200 $P --mode auto --family glm -- \
  cold_none_glm 200 $P --mode none --family glm -- \
  cold_auto_kmeans 200 $P --mode auto --family kmeans --rows 20000000 -- \
  cold_none_kmeans 200 $P --mode none --family kmeans --rows 20000000
