#!/bin/bash
# Quick GPU check of the current build: parity subset (golden fixtures, synthetic, edge cases) then a
# short bench without the CPU baseline.  tools/gpu_quick.sh OUTNAME [extra pytest -k expr]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_e2e.py -k "${2:-not table1 and not config2}" -x -q --timeout 300 --timeout-method thread > "$OUT/parity.log" 2>&1 || { tail -30 "$OUT/parity.log"; exit 1; }
tail -1 "$OUT/parity.log"
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "
import json;b=json.load(open('$OUT/bench.json'));print('value %.0f  kernel %.3f ms  ms/step %.3f' % (b['value'], b['roofline']['kernel_ms'], b['ms_per_step']))"
