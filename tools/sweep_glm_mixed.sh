#!/bin/bash
# Sweep the one-launch mixed GLM pass (grid x waves/SIMD) on the 1B x 256 bench config
# (1 GPU), with the two-stream overlap path as the control.  Results: gpurun_out/mixed_*.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_glm_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/mixed_tests.log 2>&1 || { tail -20 gpurun_out/mixed_tests.log; exit 1; }
[ -n "$NOCTL" ] || O3S_GLM_MIXED=0 timeout -k 10 180 python -u bench.py --steps 10 --warmup 2 > gpurun_out/mixed_ctl.json || exit 1
for f in ${FRACS:-0.85}; do
 for m in ${MODES:-0}; do
 for w in ${WAVES:-2 3}; do
  for g in ${GRIDS:-512 1024 2048 4096}; do
    O3S_GLM_MIX_MODE=$m O3S_GLM_MIX_WAVES=$w O3S_GLM_GRID_MIX=$g timeout -k 10 180 python -u bench.py --steps 10 \
        --warmup 2 --resident-fraction $f > gpurun_out/mixed_f${f}_m${m}_w${w}_g$g.json || exit 1
  done
 done
 done
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/mixed_*.json")):
    try:
        r = json.loads(open(f).read().strip().splitlines()[-1])
        print(f, round(r["ms_per_step"], 2), "ms", round(r["value"] / 1e9, 2), "G/s", r["final_loss"],
              r["config"]["resident_rows"])
    except Exception as e:
        print(f, "ERR", e)
PY
