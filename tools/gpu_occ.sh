#!/bin/bash
# Does a second wave per SIMD slow a chain down?  256 x 256 synthetic (TB 256: one wave per SIMD per
# workgroup) at 100 chains (one workgroup per CU) and at 512 chains (two per CU when the layout fits
# 80 KB of LDS), next to the default 256 x 512 (TB 512: two waves per SIMD).   tools/gpu_occ.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
for rep in 1 2; do
  timeout -k 10 100 python bench.py --no-cpu-baseline --steps 10 --warmup 5 > "$OUT/m512_c100_$rep.json" 2> "$OUT/m512_c100_$rep.err" || exit 1
  for c in 100 256 512; do
    timeout -k 10 150 python bench.py --no-cpu-baseline --sites 256 --taxa 256 --chains-per-gpu $c --steps 10 --warmup 5 > "$OUT/m256_c${c}_$rep.json" 2> "$OUT/m256_c${c}_$rep.err" || exit 1
  done
done
for f in "$OUT"/*.json; do python3 -c "
import json;b=json.load(open('$f'));print('%-24s %10.0f  kernel %.3f ms  lds %s' % ('$f'.split('/')[-1], b['value'], b['roofline']['kernel_ms'], b.get('config',{}).get('lds_bytes')))"; done
