#!/bin/bash
# Round 5: session warm-up -- GPU test, then the GBT config's cold vs warm fit with the
# default session (warm-up on) and with o3s.session.warmup=false.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_session_warmup.py -m gpu > gpurun_out/r5z_tests.log 2>&1 \
  || { echo "tests failed"; tail -20 gpurun_out/r5z_tests.log; exit 1; }
tail -1 gpurun_out/r5z_tests.log
timeout -k 10 400 python -u tools/bench_configs.py --config gbt --repeat 2 --out gpurun_out/r5z_gbt_default.json > gpurun_out/r5z_gbt_default.log 2>&1 \
  || { echo "gbt failed"; tail -20 gpurun_out/r5z_gbt_default.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5z_gbt_default.json')); print('default', d['fit_seconds_each'], d['session_warmup_s_untimed'], d['max_mem_gb'])"
O3S_CONF_o3s__session__warmup=false timeout -k 10 400 python -u tools/bench_configs.py --config gbt --repeat 2 --out gpurun_out/r5z_gbt_nowarm.json > gpurun_out/r5z_gbt_nowarm.log 2>&1 \
  || { echo "gbt nowarm failed"; tail -20 gpurun_out/r5z_gbt_nowarm.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5z_gbt_nowarm.json')); print('nowarm', d['fit_seconds_each'], d['session_warmup_s_untimed'])"
