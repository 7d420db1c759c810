#!/bin/bash
# Round 5: the GPU suite on the current default, the default bench line, and config 5 against a variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05l}
mkdir -p "$OUT"
V=$PWD/seriation-in-paleontological-data-using-mcmc_amd/build/var
C5="--no-cpu-baseline --parity-chains 0 --sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --warmup 5 --block-threads 1024"
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
for rep in 1 2; do
  timeout -k 10 100 python bench.py $C5 > "$OUT/c5_base_$rep.json" 2> "$OUT/c5_base_$rep.err" &&
  SERIATION_LIB=$V/${2:-nomerge}/libseriation.so timeout -k 10 100 python bench.py $C5 > "$OUT/c5_var_$rep.json" 2> "$OUT/c5_var_$rep.err" || exit 1
done
rc=$?
tail -3 "$OUT/pytest_gpu.log"
for f in "$OUT"/*.json; do python3 -c "
import json;b=json.load(open('$f'));print('%-28s %10.0f  kernel %.3f ms  tail %.2f ms' % ('$f'.split('/')[-1], b['value'], b['roofline']['kernel_ms'], b['timing']['gather_select_ms']))"; done
echo "exit $rc"
exit $rc
