cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 bash tools/debug/icache_ab.sh tools/ablibs/r3.so default tools/ablibs/sgprx.so tools/ablibs/w2bidx.so > gpurun_out/r4h_icache.txt 2>&1; echo "rc=$?"
cat gpurun_out/r4h_icache.txt
