cd $GRAFT_REPO_ROOT
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp $LIB /tmp/def.so
for L in /tmp/def.so tools/ablibs/bpw8.so tools/ablibs/bpw16.so /tmp/def.so tools/ablibs/bpw8.so tools/ablibs/bpw16.so; do
  cp $L $LIB; echo -n "$(basename $L .so): "
  timeout -k 10 90 python tools/debug/fp64_bench.py 50 || { cp /tmp/def.so $LIB; exit 1; }
done
cp /tmp/def.so $LIB
