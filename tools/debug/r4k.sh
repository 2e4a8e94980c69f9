cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_STEPS=100 timeout -k 10 900 bash tools/ab.sh tools/ablibs/r3.so tools/ablibs/v2.so tools/ablibs/v3.so tools/ablibs/v4.so tools/ablibs/v5.so tools/ablibs/v6.so tools/ablibs/r3.so tools/ablibs/v2.so tools/ablibs/v3.so tools/ablibs/v4.so tools/ablibs/v5.so tools/ablibs/v6.so > gpurun_out/r4k_ab.txt 2>&1; echo "ab rc=$?"
cat gpurun_out/r4k_ab.txt
STAMP4=1 bash tools/debug/run_stamps.sh tools/ablibs/stamp4.so tools/debug/stamps3.py > gpurun_out/r4k_stamps.txt 2>&1
