#!/bin/bash
# block-size comparison: stamps + bench at TB 256 and 512
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-tb}
mkdir -p "$OUT"
for tb in 256 512; do
  SERIATION_LIB=seriation-in-paleontological-data-using-mcmc_amd/build/stamps/libseriation.so timeout -k 10 120 python tools/stamp_profile.py tests/golden/datasets/synth_256x512.txt 100 10 $tb > "$OUT/stamps_$tb.log" 2>&1 || exit 1
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --block-threads $tb > "$OUT/bench_$tb.json" 2>"$OUT/bench_$tb.err" || exit 1
done
for tb in 256 512; do cat "$OUT/stamps_$tb.log"; cut -c1-200 "$OUT/bench_$tb.json"; done
