#!/bin/bash
# Experiment: a 256-taxon chain at TB 512 with two lanes per taxon (pair kernel, build/var/pair512)
# against one thread per taxon at TB 256, and the 512-taxon bench kernel for reference.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pair256}
mkdir -p "$OUT"
A="--no-cpu-baseline --steps 10 --warmup 10"
for rep in 1 2; do
  timeout -k 10 120 python bench.py $A --sites 256 --taxa 256 > "$OUT/t256_$rep.json" 2> "$OUT/t256_$rep.err" || exit 1
  SR_KERNEL=pair SERIATION_LIB=seriation-in-paleontological-data-using-mcmc_amd/build/var/pair512/libseriation.so \
    timeout -k 10 120 python bench.py $A --sites 256 --taxa 256 > "$OUT/p256_$rep.json" 2> "$OUT/p256_$rep.err" || exit 1
  timeout -k 10 120 python bench.py $A > "$OUT/t512_$rep.json" 2> "$OUT/t512_$rep.err" || exit 1
done
for f in "$OUT"/*.json; do python3 -c "
import json;b=json.load(open('$f'));print('%-16s %10.0f  kernel %.3f ms  %s' % ('$f'.split('/')[-1], b['value'], b['roofline']['kernel_ms'], b['config'].get('kernel')))"; done
