cd "${GRAFT_REPO_ROOT}"
bash tools/var_check.sh tools/ablibs/xw.so default tools/ablibs/xw.so default || exit 1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/b1tr -o run --output-format csv -- python3 tools/prof/batch1.py tr > gpurun_out/b1tr.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/sptr -o run --output-format csv -- python3 tools/prof/sparse_case.py > gpurun_out/sptr.log 2>&1 || exit 1
echo done
