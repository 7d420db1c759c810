#!/bin/bash
# A/B timing of the default library against build/var/<name> variants on the same box, runs
# interleaved (parity subset on the default first).   tools/gpu_ab.sh OUTNAME var1 var2 ...
# BENCH_ARGS: extra bench.py arguments (another workload, e.g. "--sites 512 --taxa 512").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
V=seriation-in-paleontological-data-using-mcmc_amd/build/var
[ -n "$NOPARITY" ] || timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py -x -q > "$OUT/parity.log" 2>&1 || { tail -20 "$OUT/parity.log"; exit 1; }
tail -1 "$OUT/parity.log"
for rep in 1 2 3; do
  timeout -k 10 100 python bench.py --no-cpu-baseline --parity-chains 0 --steps 20 --warmup 10 $BENCH_ARGS > "$OUT/base_$rep.json" 2> "$OUT/base_$rep.err" || exit 1
  for v in "$@"; do
    SERIATION_LIB=$V/$v/libseriation.so timeout -k 10 100 python bench.py --no-cpu-baseline --parity-chains 0 --steps 20 --warmup 10 $BENCH_ARGS > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || exit 1
  done
done
for f in "$OUT"/*.json; do python3 -c "
import json,sys;b=json.load(open('$f'));print('%-40s %10.0f  kernel %.3f ms' % ('$f'.split('/')[-1], b['value'], b['roofline']['kernel_ms']))"; done
