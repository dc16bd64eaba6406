#!/bin/bash
# Quick GPU check of the GLM pass: kernel + LR GPU tests, per-role timings, 1-GPU bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_glm_kernels.py tests/test_lr_gpu.py -m gpu -q -x --timeout 120 \
    --timeout-method thread > gpurun_out/glm_tests.log 2>&1 || { tail -30 gpurun_out/glm_tests.log; exit 1; }
tail -1 gpurun_out/glm_tests.log
timeout -k 10 120 python -u tools/bench_glm_roles.py --mode 0 > gpurun_out/roles_m0.json || exit 1
timeout -k 10 180 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_check.json || exit 1
python -c "
import json; r=json.load(open('gpurun_out/roles_m0.json')); print({k: round(v,2) for k,v in r.items() if not isinstance(v,str)})
r=json.loads(open('gpurun_out/bench_check.json').read().strip().splitlines()[-1]); print('bench', round(r['ms_per_step'],2), round(r['value']/1e9,2))"
