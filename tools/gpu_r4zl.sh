#!/bin/bash
# Last check of the round: the whole GPU suite and smoke() at the final defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r4zl_gputests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/r4zl_gputests.log | head -20; tail -20 gpurun_out/r4zl_gputests.log; exit 1; }
tail -1 gpurun_out/r4zl_gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4zl_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4zl_smoke.log; exit 1; }
tail -1 gpurun_out/r4zl_smoke.log
timeout -k 10 420 python -u tools/bench_configs.py --config als --iters 3 --out gpurun_out/r4zl_cfg_als.json > gpurun_out/r4zl_cfg_als.log 2>&1 || { echo "als cfg failed"; tail -30 gpurun_out/r4zl_cfg_als.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4zl_cfg_als.json')); print(d['value'], d['fit_seconds'], d['iter_seconds'])"
