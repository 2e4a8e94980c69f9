cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/debug/graph_replay.py > gpurun_out/r4e_graph.txt 2>&1; echo "graph rc=$?"; grep -c "bad archives \[\]" gpurun_out/r4e_graph.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4e_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4e_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
AB_STEPS=100 timeout -k 10 500 bash tools/ab.sh default tools/ablibs/r3.so tools/ablibs/bidx.so default tools/ablibs/r3.so tools/ablibs/bidx.so > gpurun_out/r4e_ab.txt 2>&1; echo "ab rc=$?"
cat gpurun_out/r4e_ab.txt
