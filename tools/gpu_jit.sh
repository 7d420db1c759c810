#!/bin/bash
# Shape-specialised kernels: their GPU tests, then the bench A/B (specialised vs generic) on the same box.
#   tools/gpu_jit.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-jit}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
ls -la seriation-in-paleontological-data-using-mcmc_amd/build/jit/ > "$OUT/jit_cache.txt"
for rep in 1 2 3; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 10 > "$OUT/jit_$rep.json" 2> "$OUT/jit_$rep.err" || exit 1
  timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 10 --generic > "$OUT/gen_$rep.json" 2> "$OUT/gen_$rep.err" || exit 1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --warmup 3 --block-threads 1024 > "$OUT/c5_jit.json" 2> "$OUT/c5_jit.err" || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --warmup 3 --block-threads 1024 --generic > "$OUT/c5_gen.json" 2> "$OUT/c5_gen.err" || exit 1
for f in "$OUT"/*.json; do python3 -c "
import json;b=json.load(open('$f'));print('%-14s %10.0f  kernel %.3f ms  %s %s' % ('$f'.split('/')[-1], b['value'], b['roofline']['kernel_ms'], b['config']['kernel'], b['config']['kernel_build']))"; done
