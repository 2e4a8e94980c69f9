cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 python -u tools/debug/memset_probe.py > gpurun_out/r4d_memset.txt 2>&1; echo "probe rc=$?"
timeout -k 10 120 python -u tools/debug/graph_replay.py > gpurun_out/r4c_graph.txt 2>&1; echo "graph rc=$?"
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r4c_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r4c_bench.json 2> gpurun_out/r4c_bench.err || exit 1
head -c 1200 gpurun_out/r4c_bench.json
