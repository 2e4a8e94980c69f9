cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/debug/graph_replay.py > gpurun_out/r4b_graph.txt 2>&1; echo "graph rc=$?"
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4b_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/r4b_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python bench.py > gpurun_out/r4b_bench.json 2> gpurun_out/r4b_bench.err || exit 1
head -c 1500 gpurun_out/r4b_bench.json
bash tools/debug/run_stamps.sh tools/ablibs/stamp3.so tools/debug/stamps3.py > gpurun_out/r4b_stamps.txt 2>&1
