cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_STEPS=100 timeout -k 10 900 bash tools/ab.sh tools/ablibs/r3.so tools/ablibs/v9.so tools/ablibs/v7.so tools/ablibs/plainpart.so tools/ablibs/plainall.so tools/ablibs/v8.so tools/ablibs/v2.so tools/ablibs/r3.so tools/ablibs/v9.so tools/ablibs/v7.so tools/ablibs/plainpart.so tools/ablibs/plainall.so tools/ablibs/v8.so tools/ablibs/v2.so > gpurun_out/r4l_ab.txt 2>&1; echo "ab rc=$?"
cat gpurun_out/r4l_ab.txt
