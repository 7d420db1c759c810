#!/bin/bash
# Config 5 (1024 x 2048, split chains): parity of the split / HBM-column paths on the current build, then the
# config-5 bench of the current build against build/var/<old>, interleaved on one box.
#   tools/gpu_c5_lck.sh OUTNAME OLDVAR [REPS]     (WARM="3 100": warm-up launches of each A/B pair; default 10)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; OLD=$2; REPS=${3:-3}
mkdir -p "$OUT"
V=seriation-in-paleontological-data-using-mcmc_amd/build/var
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_config5.py -k "hbm or per-thread or tb1024 or n2500 or config5 or split" -x -v --timeout 300 --timeout-method thread > "$OUT/parity.log" 2>&1 || { tail -30 "$OUT/parity.log"; exit 1; }
tail -1 "$OUT/parity.log"
C5="--sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --parity-chains 0"
for w in ${WARM:-10}; do
for rep in $(seq 1 $REPS); do
  timeout -k 10 200 python bench.py --no-cpu-baseline $C5 --warmup $w > "$OUT/c5new_w${w}_$rep.json" 2> "$OUT/c5new_w${w}_$rep.err" || exit 1
  SERIATION_LIB=$V/$OLD/libseriation.so timeout -k 10 200 python bench.py --no-cpu-baseline $C5 --warmup $w > "$OUT/c5old_w${w}_$rep.json" 2> "$OUT/c5old_w${w}_$rep.err" || exit 1
done
done
for f in "$OUT"/c5*.json; do python3 -c "
import json;b=json.load(open('$f'));print('%-24s %10.0f  kernel %.3f ms' % ('$f'.split('/')[-1], b['value'], b['roofline']['kernel_ms']))"; done
