#!/bin/bash
# SQ issue/park split and instruction counts of the pair kernel and the single kernel on the bench
# workload (one --pmc run per pass and kernel).   tools/gpu_sq_ab.sh OUTNAME
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
P="bench.py --no-cpu-baseline --steps 5 --warmup 3"
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
SQB="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_INSTS_VMEM SQ_INSTS_BRANCH"
for k in pair single; do
  E="SR_KERNEL=$k"
  env $E timeout -s KILL 180 rocprofv3 --pmc $SQA --output-format csv -d "$OUT/${k}_sq" -o s -- python3 $P > "$OUT/${k}_sq.log" 2>&1 || exit 1
  env $E timeout -s KILL 180 rocprofv3 --pmc $SQB --output-format csv -d "$OUT/${k}_sq_b" -o s -- python3 $P > "$OUT/${k}_sq_b.log" 2>&1 || exit 1
done
echo done
