#!/bin/bash
# Config 5's L2 behaviour against the chain count: TCC_HIT / TCC_MISS and FETCH_SIZE passes (separate runs, ordinary
# launch as every config-5 PMC pass) at 16, 32, 64 and 100 chains, 10 warm-up launches of 2 calls, 10 timed.
#   tools/gpu_c5_l2.sh NAME  ->  gpurun_out/NAME/l2_n<chains>/, fetch_n<chains>/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp SR_COOP=0
OUT=gpurun_out/${1:-c5l2}
mkdir -p "$OUT"
C5="bench.py --no-cpu-baseline --legs none --parity-chains 0 --sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --warmup 10 --block-threads 1024"
for n in ${CHAINS:-16 32 64 100}; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/l2_n$n" -o h -- python3 $C5 --total-chains $n > "$OUT/l2_n$n.log" 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_n$n" -o f -- python3 $C5 --total-chains $n > "$OUT/fetch_n$n.log" 2>&1 || exit 1
  echo "chains $n done"
done
echo done
