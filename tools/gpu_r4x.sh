#!/bin/bash
# KMeans update kernel at 2 and 3 blocks per CU (100M x 128, k 1024 / 64); the slab-flush
# variants timed with it are recorded in profiles/kernel_experiments_r4.json
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_kmeans_update.py --ks 1024,64 --iters 10 > gpurun_out/r4x_update_g512.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_kmeans_update.py --ks 1024,64 --iters 10 --grid 768 > gpurun_out/r4x_update_g768.log 2>&1
