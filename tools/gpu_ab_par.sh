#!/bin/bash
# A/B with a parity check of every variant: tests/test_gpu_parity.py on each build/var/<name> library first
# (the variants change kernel logic, not only timing), then bench.py of the default library and the variants
# interleaved, 3 rounds.   tools/gpu_ab_par.sh OUTNAME var1 var2 ...   (BENCH_ARGS: extra bench.py arguments)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
V=seriation-in-paleontological-data-using-mcmc_amd/build/var
timeout -k 10 300 python -m pytest ${PARITY:-tests/test_gpu_parity.py} -x -q -p no:cacheprovider > "$OUT/parity_default.log" 2>&1 ||
  { tail -30 "$OUT/parity_default.log"; exit 1; }
echo "default: $(tail -1 "$OUT/parity_default.log")"
for v in "$@"; do
  SERIATION_LIB=$PWD/$V/$v/libseriation.so timeout -k 10 300 python -m pytest ${PARITY:-tests/test_gpu_parity.py} -x -q \
    -p no:cacheprovider > "$OUT/parity_$v.log" 2>&1 || { tail -30 "$OUT/parity_$v.log"; exit 1; }
  echo "$v: $(tail -1 "$OUT/parity_$v.log")"
done
for rep in 1 2 3; do
  timeout -k 10 100 python bench.py --no-cpu-baseline --parity-chains 0 --steps 20 --warmup 10 $BENCH_ARGS > "$OUT/base_$rep.json" 2> "$OUT/base_$rep.err" || exit 1
  for v in "$@"; do
    SERIATION_LIB=$PWD/$V/$v/libseriation.so timeout -k 10 100 python bench.py --no-cpu-baseline --parity-chains 0 --steps 20 --warmup 10 $BENCH_ARGS > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || exit 1
  done
done
for f in "$OUT"/*.json; do python3 -c "
import json,sys;b=json.load(open('$f'));print('%-40s %10.0f  kernel %.3f ms  %s' % ('$f'.split('/')[-1], b['value'], b['roofline']['kernel_ms'], b['config']['kernel_build']))"; done
