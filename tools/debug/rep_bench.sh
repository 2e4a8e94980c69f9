cd "${GRAFT_REPO_ROOT}"
for i in 1 2 3 4 5 6; do
  DIETGPU_BENCH_ADDRS=1 timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extras --steps 100 --warmup 5 > gpurun_out/rep_$i.log 2> gpurun_out/rep_$i.err || exit 1
  python3 -c "
import json
for l in open('gpurun_out/rep_$i.log'):
    if l.startswith('{'):
        d=json.loads(l); print($i, d['ms_per_step'], d['kernels'])
for l in open('gpurun_out/rep_$i.err'):
    if l.startswith('addrs'): print(l.strip())"
done
