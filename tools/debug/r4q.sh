cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_grid.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "sparse or float_stride or fp64" > gpurun_out/r4q_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4q_tests.log
[ $rc -eq 0 ] || exit $rc
cp dietgpu_fork_amd/_lib/libdietgpu_amd.so /tmp/kt2.so
timeout -k 10 300 bash tools/debug/sp_ab.sh /tmp/kt2.so tools/ablibs/kt1.so /tmp/kt2.so tools/ablibs/kt1.so
