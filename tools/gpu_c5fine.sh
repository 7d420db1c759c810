#!/bin/bash
# Config 5 at TB 512 (4 taxa per thread) next to TB 1024, and the fine stamp split of the TB-512 run
# (SR_STAMP_FINE supports <= 8 waves).   tools/gpu_c5fine.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
C5="--sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --warmup 3"
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline $C5 --block-threads 1024 > "$OUT/tb1024_$rep.json" 2> "$OUT/tb1024_$rep.err" || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline $C5 --block-threads 512 > "$OUT/tb512_$rep.json" 2> "$OUT/tb512_$rep.err" || exit 1
done
DS=$(ls /tmp/sr_synth_1024x2048_*.txt | head -1)
SR_FINE=1 SERIATION_LIB=seriation-in-paleontological-data-using-mcmc_amd/build/var/fine/libseriation.so timeout -k 10 200 python tools/stamp_profile.py "$DS" 100 2 512 > "$OUT/fine512.txt" 2>&1 || exit 1
cat "$OUT/fine512.txt"
for f in "$OUT"/*.json; do python3 -c "
import json;b=json.load(open('$f'));print('%-24s %10.0f  kernel %.3f ms' % ('$f'.split('/')[-1], b['value'], b['roofline']['kernel_ms']))"; done
