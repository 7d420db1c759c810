#!/bin/bash
# Config 5 (1024 x 2048, split chains) for the round record: its bench line, the kernel trace of the
# same command and separate FETCH / WRITE / SQ --pmc passes.  The profiled runs launch the split
# grid without the cooperative API (SR_COOP=0: rocprofv3's tracer crashes at exit after cooperative
# launches, gpurun_out/r03w/c5_prof.log); the bench line itself is the default (cooperative) launch.
# plus an L2 hit / miss pass (TCC_HIT_sum, TCC_MISS_sum).
#   tools/gpu_c5_round.sh NAME  ->  tools/pmc_summary.py gpurun_out/NAME profiles/NAME_config5 --tag c5_
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-c5round}
mkdir -p "$OUT"
C5="bench.py --no-cpu-baseline --sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --warmup 3 --block-threads 1024"
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
SQB="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"
timeout -k 10 200 python $C5 > "$OUT/c5_bench.json" 2> "$OUT/c5_bench.err" &&
SR_COOP=0 timeout -k 10 200 python $C5 > "$OUT/c5_bench_nocoop.json" 2> "$OUT/c5_bench_nocoop.err" &&
SR_COOP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5_prof" -o c5 -- python3 $C5 > "$OUT/c5_prof.log" 2>&1 &&
SR_COOP=0 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/c5_fetch" -o f -- python3 $C5 > "$OUT/c5_fetch.log" 2>&1 &&
SR_COOP=0 timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/c5_write" -o w -- python3 $C5 > "$OUT/c5_write.log" 2>&1 &&
SR_COOP=0 timeout -s KILL 180 rocprofv3 --pmc $SQA --output-format csv -d "$OUT/c5_sq" -o s -- python3 $C5 > "$OUT/c5_sq.log" 2>&1 &&
SR_COOP=0 timeout -s KILL 180 rocprofv3 --pmc $SQB --output-format csv -d "$OUT/c5_sq_b" -o s -- python3 $C5 > "$OUT/c5_sq_b.log" 2>&1 &&
SR_COOP=0 timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/c5_l2" -o l -- python3 $C5 > "$OUT/c5_l2.log" 2>&1
rc=$?
echo "exit $rc"
exit $rc
