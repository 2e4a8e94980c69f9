for L in cur lb4 cur lb4; do cp tools/ablibs/$L.so dietgpu_fork_amd/_lib/libdietgpu_amd.so; echo -n "$L: "; timeout -k 10 60 python tools/debug/sparse_bench.py 50 || exit 1; done
cp tools/ablibs/lb4.so dietgpu_fork_amd/_lib/libdietgpu_amd.so
