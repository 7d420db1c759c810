#!/bin/bash
# Where a sweep's wave-cycles go: SQ issue/park split of the bench kernel (config 3) and the HBM
# traffic + SQ counters of config 5 (1024 x 2048, HBM columns), each --pmc pass a run of its own,
# timed launches only.   tools/gpu_probe.sh OUTNAME
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-probe}
mkdir -p "$OUT"
B="bench.py --no-cpu-baseline --steps 5 --warmup 3"
C5="bench.py --no-cpu-baseline --sites 1024 --taxa 2048 --calls-per-step 2 --steps 5 --warmup 3 --block-threads 1024"
# a step that ends in a signal, a time limit or an abort ends the script; an ordinary failure
# (e.g. a counter this rocprofv3 does not know) is recorded and the next step runs
step() {
  local name=$1; shift
  "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step list timeout -s KILL 60 rocprofv3 -L
step sq_a timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA --output-format csv -d "$OUT/sq_a" -o a -- python3 $B
step sq_b timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC --output-format csv -d "$OUT/sq_b" -o b -- python3 $B
step sq_c timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT --output-format csv -d "$OUT/sq_c" -o c -- python3 $B
step c5_trace timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5_prof" -o c5 -- python3 $C5
step c5_fetch timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/c5_fetch" -o f -- python3 $C5
step c5_write timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/c5_write" -o w -- python3 $C5
step c5_sq timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d "$OUT/c5_sq" -o s -- python3 $C5
step c5_tcp timeout -s KILL 180 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/c5_tcp" -o t -- python3 $C5
echo done
