#!/bin/bash
# The pair kernel (two lanes per taxon) against the one-thread-per-taxon kernel in the same build
# (SR_KERNEL=single, the default), same box, runs interleaved; the parity subset runs on the pair kernel first.
#   tools/gpu_pair_ab.sh OUTNAME [pytest -k expr]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
SR_KERNEL=pair timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py -x -q --timeout 300 --timeout-method thread -k "${2:-not reference_protocol}" > "$OUT/parity.log" 2>&1 || { tail -30 "$OUT/parity.log"; exit 1; }
tail -1 "$OUT/parity.log"
for rep in 1 2 3; do
  SR_KERNEL=pair timeout -k 10 100 python bench.py --no-cpu-baseline --steps 20 --warmup 10 > "$OUT/pair_$rep.json" 2> "$OUT/pair_$rep.err" || { tail "$OUT/pair_$rep.err"; exit 1; }
  SR_KERNEL=single timeout -k 10 100 python bench.py --no-cpu-baseline --steps 20 --warmup 10 > "$OUT/single_$rep.json" 2> "$OUT/single_$rep.err" || exit 1
done
for f in "$OUT"/*.json; do python3 -c "
import json;b=json.load(open('$f'));print('%-30s %10.0f  kernel %.3f ms  tb %d' % ('$f'.split('/')[-1], b['value'], b['roofline']['kernel_ms'], b['config']['block_threads']))"; done
