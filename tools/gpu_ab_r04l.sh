#!/bin/bash
# Round-4 experiment: config 5 on 512-thread split halves with two taxa per thread (SR_SPLIT=2, 256 VGPRs, no
# spills) against the product's 1024-thread halves (one taxon per thread, 128 VGPRs).  Parity first
# (tools/sp512_check.py), then interleaved bench runs.   tools/gpu_ab_r04l.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04l}
mkdir -p $OUT
SR_SPLIT=2 timeout -k 10 300 python tools/sp512_check.py > $OUT/sp512_parity.json 2> $OUT/sp512_parity.err || { cat $OUT/sp512_parity.json; tail -5 $OUT/sp512_parity.err; exit 1; }
cat $OUT/sp512_parity.json
C5="--no-cpu-baseline --parity-chains 0 --steps 20 --warmup 10 --sites 1024 --taxa 2048 --calls-per-step 2"
for rep in 1 2 3; do
  timeout -k 10 100 python bench.py $C5 --block-threads 1024 > $OUT/base_$rep.json 2> $OUT/base_$rep.err || exit 1
  SR_SPLIT=2 timeout -k 10 100 python bench.py $C5 --block-threads 512 > $OUT/sp512_$rep.json 2> $OUT/sp512_$rep.err || exit 1
done
for f in $OUT/*_[123].json; do python3 -c "
import json;b=json.load(open('$f'));print('%-16s %10.0f  kernel %.3f ms  %s %s' % ('$f'.split('/')[-1], b['value'], b['roofline']['kernel_ms'], b['config']['kernel'], b['config']['block_threads']))"; done
