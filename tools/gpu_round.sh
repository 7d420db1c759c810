#!/bin/bash
# One full GPU-box pass for the round record: smoke, GPU test suite, the default bench (CPU
# baseline included), rocprofv3 --kernel-trace --stats of that SAME bench command, separate --pmc
# passes (HBM FETCH_SIZE / WRITE_SIZE, SQ/LDS counters) over it, then config 5 (1024 x 2048, HBM
# columns) with its own kernel trace.  Every GPU step has its own time limit; the chain stops at the
# first failure.   tools/gpu_round.sh NAME   ->  tools/pmc_summary.py gpurun_out/NAME profiles/NAME
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-round}
mkdir -p "$OUT"
B="bench.py"
C5="bench.py --no-cpu-baseline --sites 1024 --taxa 2048 --calls-per-step 2 --steps 5 --warmup 3 --block-threads 1024"
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python $B > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 $B > "$OUT/prof.log" 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o f -- python3 $B --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o w -- python3 $B --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d "$OUT/pmc_sq" -o s -- python3 $B --no-cpu-baseline > "$OUT/pmc_sq.log" 2>&1 &&
timeout -k 10 200 python $C5 > "$OUT/c5_bench.json" 2> "$OUT/c5_bench.err" &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5_prof" -o c5 -- python3 $C5 > "$OUT/c5_prof.log" 2>&1
rc=$?
echo "exit $rc"
exit $rc
