#!/bin/bash
# A/B sweep of the GLM pass launch shape (overlap on/off, resident / lineage grids) through bench.py
set -o pipefail
run() { echo "== $1" >> gpurun_out/sweep_overlap.log; env $2 timeout -k 10 180 python bench.py --steps 20 --warmup 3 >> gpurun_out/sweep_overlap.log 2>&1; }
run A "O3S_GLM_OVERLAP=0" && run B "O3S_GLM_OVERLAP=1" && run C "O3S_GLM_GRID_RES=768 O3S_GLM_GRID_LIN=256" && run D "O3S_GLM_GRID_RES=512 O3S_GLM_GRID_LIN=512" && run E "O3S_GLM_GRID_RES=2048 O3S_GLM_GRID_LIN=256" && run F "O3S_GLM_GRID_RES=1024 O3S_GLM_GRID_LIN=512"
