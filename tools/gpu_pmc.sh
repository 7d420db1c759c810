#!/bin/bash
# PMC passes over the bench workload (separate --pmc runs, kernel-trace only; no sys/runtime trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc}
mkdir -p "$OUT"
B="bench.py --no-cpu-baseline --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$OUT/p1" -o p1 -- python3 $B > "$OUT/p1.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA --output-format csv -d "$OUT/p2" -o p2 -- python3 $B > "$OUT/p2.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$OUT/p3" -o p3 -- python3 $B > "$OUT/p3.log" 2>&1
rc=$?
find "$OUT" -name "*counter_collection.csv" | head
exit $rc
