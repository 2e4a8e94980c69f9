#!/bin/bash
# GPU box: parity-checked same-box A/B of kernel-variant libraries.  Each
# variant is swapped in, its oracle/golden parity tests run once, then the
# c2 bench (with the cold/warm decode probe) runs PASSES times, alternating
# libraries per pass.  The in-tree library is restored after.
#   usage: PASSES=2 bash tools/ab2.sh default tools/ablibs/x.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/ab2_default.so
trap 'cp /tmp/ab2_default.so "$LIB"' EXIT
swap() { if [ "$1" = default ]; then cp /tmp/ab2_default.so "$LIB"; else cp "$1" "$LIB"; fi; }
if [ -z "$NO_PARITY" ]; then
  for L in "$@"; do
    [ "$L" = default ] && continue
    T=$(basename "$L" .so)
    swap "$L"
    timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_compress_paths.py tests/test_gpu_teams.py} \
      -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab2_$T.log 2>&1 \
      || { echo "$T parity FAILED"; tail -30 gpurun_out/ab2_$T.log; exit 1; }
    echo "$T parity $(tail -1 gpurun_out/ab2_$T.log)"
  done
fi
for p in $(seq 1 ${PASSES:-2}); do
  for L in "$@"; do
    T=$(basename "$L" .so)
    swap "$L"
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --no-verify --steps ${AB_STEPS:-100} \
      > gpurun_out/ab2_${T}_$p.log 2>&1 || { echo "$T bench FAILED"; tail -5 gpurun_out/ab2_${T}_$p.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/ab2_${T}_$p.log'):
    if l.startswith('{'):
        d = json.loads(l); h = d.get('decode_hbm') or {}
        print('pass $p', '$T', d['value'], d['ms_per_step'], d['kernels'], 'dec warm/cold', h.get('decode_warm_ms'), h.get('decode_cold_ms'), 'step cold', h.get('step_cold_ms'))"
  done
done
