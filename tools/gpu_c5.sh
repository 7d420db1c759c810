#!/bin/bash
# Config 5 (1024 x 2048, HBM columns): parity of the HBM-column / several-taxa-per-thread paths, then
# the config-5 bench at 1024 and 512 threads for the current build and build/var/<old>, then the
# SR_STAMPS phase split (build/var/stamps).   tools/gpu_c5.sh OUTNAME OLDVAR
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; OLD=$2
mkdir -p "$OUT"
V=seriation-in-paleontological-data-using-mcmc_amd/build/var
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_config5.py -k "hbm or per-thread or tb1024 or n2500 or config5" -x -q --timeout 300 --timeout-method thread > "$OUT/parity.log" 2>&1 || { tail -30 "$OUT/parity.log"; exit 1; }
tail -1 "$OUT/parity.log"
C5="--sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --warmup 3"
for tb in 1024 512; do
  timeout -k 10 200 python bench.py --no-cpu-baseline $C5 --block-threads $tb > "$OUT/c5new_$tb.json" 2> "$OUT/c5new_$tb.err" || exit 1
  SERIATION_LIB=$V/$OLD/libseriation.so timeout -k 10 200 python bench.py --no-cpu-baseline $C5 --block-threads $tb > "$OUT/c5old_$tb.json" 2> "$OUT/c5old_$tb.err" || exit 1
done
for f in "$OUT"/*.json; do python3 -c "
import json;b=json.load(open('$f'));print('%-24s %10.0f  kernel %.3f ms' % ('$f'.split('/')[-1], b['value'], b['roofline']['kernel_ms']))"; done
for tb in 1024 512; do
  SERIATION_LIB=$V/stamps/libseriation.so timeout -k 10 200 python tools/stamp_profile.py /tmp/sr_synth_1024x2048_20261016.txt 100 2 $tb > "$OUT/stamps_$tb.txt" 2>&1 || exit 1
  cat "$OUT/stamps_$tb.txt"
done
