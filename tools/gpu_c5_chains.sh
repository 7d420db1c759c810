#!/bin/bash
# Config 5 (1024 x 2048, split chains, cooperative launch) against the chain count on one GPU: is the launch time
# set by the per-XCD working set (L2 4 MB per XCD; ~220 KB of columns, prefixes and state per half-chain) or by
# the chain's own latency?  10 warm-up launches of 2 calls, 10 timed, interleaved x2.
#   tools/gpu_c5_chains.sh NAME  ->  gpurun_out/NAME/c5_n<chains>_<rep>.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-c5chains}
mkdir -p "$OUT"
C5="bench.py --no-cpu-baseline --legs none --parity-chains 0 --sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --warmup 10 --block-threads 1024"
for rep in 1 2; do
  for n in ${CHAINS:-8 16 32 64 100 128}; do
    timeout -k 10 200 python $C5 --total-chains $n > "$OUT/c5_n${n}_$rep.json" 2> "$OUT/c5_n${n}_$rep.err" || exit 1
    python3 -c "
import json;b=json.load(open('$OUT/c5_n${n}_$rep.json'));print('%4d chains: %8.0f chain-iter/s  kernel %.3f ms  %s' % ($n, b['value'], b['roofline']['kernel_ms'], b['config'].get('launch')))"
  done
done
echo done
