#!/bin/bash
# Parity of the current build on the kernels a change touches, then config 3 and config 5 benches of
# the current build against build/var/<old> (interleaved, same box).
#   tools/gpu_check.sh OUTNAME OLDVAR [pytest files...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; OLD=$2; shift 2
mkdir -p "$OUT"
V=seriation-in-paleontological-data-using-mcmc_amd/build/var
T=${*:-tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_config5.py tests/test_gpu_fallbacks.py}
timeout -k 10 600 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread > "$OUT/parity.log" 2>&1 || { tail -30 "$OUT/parity.log"; exit 1; }
tail -1 "$OUT/parity.log"
C5="--sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --warmup 3 --block-threads 1024"
for rep in 1 2; do
  timeout -k 10 100 python bench.py --no-cpu-baseline --steps 20 --warmup 10 > "$OUT/new_$rep.json" 2> "$OUT/new_$rep.err" || exit 1
  SERIATION_LIB=$V/$OLD/libseriation.so timeout -k 10 100 python bench.py --no-cpu-baseline --steps 20 --warmup 10 > "$OUT/old_$rep.json" 2> "$OUT/old_$rep.err" || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline $C5 > "$OUT/c5new_$rep.json" 2> "$OUT/c5new_$rep.err" || exit 1
  SERIATION_LIB=$V/$OLD/libseriation.so timeout -k 10 200 python bench.py --no-cpu-baseline $C5 > "$OUT/c5old_$rep.json" 2> "$OUT/c5old_$rep.err" || exit 1
done
for f in "$OUT"/*.json; do python3 -c "
import json;b=json.load(open('$f'));print('%-24s %10.0f  kernel %.3f ms' % ('$f'.split('/')[-1], b['value'], b['roofline']['kernel_ms']))"; done
