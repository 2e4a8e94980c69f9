cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_STEPS=100 timeout -k 10 900 bash tools/ab.sh tools/ablibs/r3.so tools/ablibs/v14.so tools/ablibs/v13.so tools/ablibs/v11.so tools/ablibs/v12.so tools/ablibs/r3.so tools/ablibs/v14.so tools/ablibs/v13.so tools/ablibs/v11.so tools/ablibs/v12.so > gpurun_out/r4m_ab.txt 2>&1; echo "ab rc=$?"
cat gpurun_out/r4m_ab.txt
