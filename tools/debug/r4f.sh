cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_STEPS=100 timeout -k 10 500 bash tools/ab.sh tools/ablibs/r3.so tools/ablibs/bidx0.so tools/ablibs/sgprx.so tools/ablibs/r3.so tools/ablibs/bidx0.so tools/ablibs/sgprx.so > gpurun_out/r4f_ab.txt 2>&1; echo "ab rc=$?"
cat gpurun_out/r4f_ab.txt
