#!/bin/bash
# Rehearse the N = 2 shape of the scaling run on ONE GPU: 2 ranks over gloo, each holding
# HBM-resident rows AND rows regenerated in-kernel from lineage (small resident fraction),
# against one rank on the same 200M x 256 table -- the loss curves must agree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O3S_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 1 --rows 200000000 \
    --resident-fraction 0.08 --rehearsal --no-hbm-only > gpurun_out/lineage_n2.json 2> gpurun_out/lineage_n2.err \
  || { tail -30 gpurun_out/lineage_n2.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --rows 200000000 --resident-fraction 0.08 --no-hbm-only \
    > gpurun_out/lineage_n1.json 2> gpurun_out/lineage_n1.err || { tail -30 gpurun_out/lineage_n1.err; exit 1; }
grep -v amdgpu.ids gpurun_out/lineage_n2.json; grep -v amdgpu.ids gpurun_out/lineage_n1.json
