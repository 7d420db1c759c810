#!/bin/bash
# GPU tests given as arguments, then three default bench lines.   tools/gpu_quick_bench.sh OUT tests...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for rep in 1 2 3; do
  timeout -k 10 150 python bench.py --no-cpu-baseline > "$OUT/bench_$rep.json" 2> "$OUT/bench_$rep.err" || exit 1
done
for f in "$OUT"/bench_*.json; do python3 -c "
import json;b=json.load(open('$f'));print('%-14s %10.0f  ms/step %.3f kernel %.3f ms  tail %.2f ms  %s' % ('$f'.split('/')[-1], b['value'], b['ms_per_step'], b['roofline']['kernel_ms'], b['timing']['gather_select_ms'], b['config']['kernel_build'])); print(b['timing']['tail_parts'])"; done
