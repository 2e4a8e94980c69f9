cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ds.log 2>&1 || { tail -30 gpurun_out/t_ds.log; exit 1; }
tail -1 gpurun_out/t_ds.log
NO_PARITY=1 bash tools/var_check.sh tools/ablibs/cur.so tools/ablibs/dstart.so tools/ablibs/cur.so tools/ablibs/dstart.so || exit 1
bash tools/debug/extras_ab.sh tools/ablibs/cur.so tools/ablibs/dstart.so
