#!/bin/bash
# Round 6, second box pass (after the planner change): smoke, the whole GPU suite, the default bench line, then
# the measurements the review asked about:
#   - threads per chain: 256 x 512 at 512 threads (one taxon per thread, 8 waves per chain: the product) against
#     256 threads (two taxa per thread, 4 waves) -- the direction of north_star's "one wavefront per chain";
#   - the metric at N = 8's per-GPU load: 13 chains on one GPU (13/13/13/13/12/12/12/12 at N = 8);
#   - config 4's 800 chains on one GPU (the strong-scaling form's N = 1 point);
#   - config 1: the product CLI on g2s2 (1 chain, CLI defaults: 1000 + 1000 calls), wall time.
# Each GPU step has its own limit; the chain stops at the first failure.     tools/gpu_r06d.sh NAME
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06d}
mkdir -p "$OUT"
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 500 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
Q="--legs none --no-cpu-baseline --parity-chains 2 --parity-rejected 0 --parity-calls 20"
for rep in 1 2; do
  for tb in 512 256; do
    timeout -k 10 200 python bench.py $Q --block-threads $tb > "$OUT/tb${tb}_$rep.json" 2> "$OUT/tb${tb}_$rep.err" || exit 1
  done
done
timeout -k 10 200 python bench.py $Q --total-chains 13 > "$OUT/chains13.json" 2> "$OUT/chains13.err" || exit 1
timeout -k 10 300 python bench.py $Q --total-chains 800 > "$OUT/chains800.json" 2> "$OUT/chains800.err" || exit 1
D=$(mktemp -d) && mkdir -p "$D/Chains/chain_00" && CLI=$PWD/seriation-in-paleontological-data-using-mcmc_amd/build/mcmc &&
( cd "$D" && s=$(date +%s.%N) && GSL_RNG_SEED=1 timeout -k 10 120 "$CLI" 0 < "$OLDPWD/tests/golden/datasets/g2s2.txt" > /dev/null 2> cli.err &&
  e=$(date +%s.%N) && python3 -c "print('{\"config1_cli_wall_s\": %.3f}' % ($e - $s))" ) > "$OUT/config1.json" || exit 1
for f in "$OUT"/tb*.json "$OUT"/chains*.json; do python3 -c "
import json;b=json.load(open('$f'));print('%-18s %10.0f chain-iter/s  kernel %.3f ms  chains %d' % ('$f'.split('/')[-1], b['value'], b['roofline']['kernel_ms'], b['config']['chains']))"; done
cat "$OUT/config1.json"
echo done
