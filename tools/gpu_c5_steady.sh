#!/bin/bash
# Config 5 (1024 x 2048, 100 chains, split chains) against chain age: bench lines after 3 .. 500 warm-up launches
# (2 calls = 20 sweeps each; 500 launches = the headline's 1000 warm-up calls), then the SQ issue / park pass
# over a run with 100 warm-up launches (ordinary launch, SR_COOP=0, as every config-5 profile).
#   tools/gpu_c5_steady.sh NAME  ->  tools/pmc_summary.py gpurun_out/NAME profiles/NAME --tag c5_ --warmup 100 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-c5steady}
mkdir -p "$OUT"
C5="bench.py --no-cpu-baseline --parity-chains 0 --sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --block-threads 1024"
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
for w in 3 10 30 100 250 500; do
  timeout -k 10 200 python $C5 --warmup $w > "$OUT/c5_w$w.json" 2> "$OUT/c5_w$w.err" || exit 1
  python3 -c "
import json;b=json.load(open('$OUT/c5_w$w.json'));print('warmup %4d launches: %8.0f chain-iter/s  kernel %.3f ms' % ($w, b['value'], b['roofline']['kernel_ms']))"
done
SR_COOP=0 timeout -k 10 200 python $C5 --warmup 100 > "$OUT/c5_bench.json" 2> "$OUT/c5_bench.err" &&
SR_COOP=0 timeout -s KILL 180 rocprofv3 --pmc $SQA --output-format csv -d "$OUT/c5_sq" -o s -- python3 $C5 --warmup 100 > "$OUT/c5_sq.log" 2>&1 &&
SR_COOP=0 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/c5_fetch" -o f -- python3 $C5 --warmup 100 > "$OUT/c5_fetch.log" 2>&1 &&
SR_COOP=0 timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/c5_write" -o w -- python3 $C5 --warmup 100 > "$OUT/c5_write.log" 2>&1 &&
SR_COOP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5_prof" -o c5 -- python3 $C5 --warmup 100 > "$OUT/c5_prof.log" 2>&1
rc=$?
echo "exit $rc"
exit $rc
