#!/bin/bash
# Rehearse the multi-rank bench path on ONE GPU (2 ranks over gloo, small table) and
# time one rank's share of the N=8 run (125M x 256 rows, all HBM-resident).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O3S_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --rows 100000000 --rehearsal \
    > gpurun_out/rehearsal_n2.json 2> gpurun_out/rehearsal_n2.err || { tail -30 gpurun_out/rehearsal_n2.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --rows 125000000 > gpurun_out/share_n8.json || exit 1
grep -v amdgpu.ids gpurun_out/rehearsal_n2.json; grep -v amdgpu.ids gpurun_out/share_n8.json
