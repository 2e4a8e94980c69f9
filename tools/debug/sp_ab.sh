for L in cur rts cur rts; do cp tools/ablibs/$L.so dietgpu_fork_amd/_lib/libdietgpu_amd.so; echo -n "$L: "; timeout -k 10 60 python tools/debug/sparse_bench.py 50 || exit 1; done
cp tools/ablibs/rts.so dietgpu_fork_amd/_lib/libdietgpu_amd.so
