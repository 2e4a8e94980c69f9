cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 python -u tools/debug/memset_probe.py > gpurun_out/r4d_memset.txt 2>&1; echo "probe rc=$?"
cat gpurun_out/r4d_memset.txt
AB_STEPS=100 timeout -k 10 500 bash tools/ab.sh default tools/ablibs/r3.so tools/ablibs/bidx.so default tools/ablibs/r3.so tools/ablibs/bidx.so > gpurun_out/r4d_ab.txt 2>&1; echo "ab rc=$?"
cat gpurun_out/r4d_ab.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > gpurun_out/r4d_bench.json 2> gpurun_out/r4d_bench.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/r4d_bench.json').read().splitlines()[0]); print(d['value'], d['kernels'], json.dumps(d.get('decode_hbm')))"
