for g in 1 2 4; do
O3S_HIST_G=$g timeout -k 10 300 python -u -m pytest tests/test_trees.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/trees_test.log 2>&1 || { tail -30 gpurun_out/trees_test.log; exit 1; }
echo "G=$g $(tail -1 gpurun_out/trees_test.log)"
O3S_HIST_G=$g timeout -k 10 120 python -u tools/bench_hist.py 2>/dev/null | tail -1
O3S_HIST_G=$g timeout -k 10 200 python -u tools/bench_gbt.py --trees 3 2>/dev/null | tail -1 | cut -c1-110
done
