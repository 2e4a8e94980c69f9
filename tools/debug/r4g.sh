cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compress_paths.py tests/test_gpu_progress.py tests/test_gpu_golden.py tests/test_gpu_api.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r4g_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4g_tests.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=100 timeout -k 10 700 bash tools/ab.sh tools/ablibs/r3.so default tools/ablibs/w2bidx.so tools/ablibs/bidx0.so tools/ablibs/sgprx.so tools/ablibs/r3.so default tools/ablibs/w2bidx.so tools/ablibs/bidx0.so tools/ablibs/sgprx.so > gpurun_out/r4g_ab.txt 2>&1; echo "ab rc=$?"
cat gpurun_out/r4g_ab.txt
