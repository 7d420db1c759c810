#!/bin/bash
# One full GPU-box pass for the round record: smoke, GPU test suite, the default bench (CPU
# baseline and the config2 / config5 legs included), rocprofv3 --kernel-trace --stats of the headline bench command
# (--legs none --no-cpu-baseline: the same timed workload, without the legs' other kernels), separate --pmc
# passes over it (HBM FETCH_SIZE / WRITE_SIZE; SQ issue / park split, instruction mix, LDS), then
# config 5 (1024 x 2048, HBM columns) with its own bench line (after 3 warm-up launches, and after 100 = 2000
# sweeps: c5_bench_ss, nearer the steady state of the headline's 1000 warm-up calls), kernel trace and FETCH / WRITE / SQ
# passes.  Every GPU step has its own time limit; the chain stops at the first failure.
#   tools/gpu_round.sh NAME [skip-tests]  ->  tools/pmc_summary.py gpurun_out/NAME profiles/NAME
#                                            tools/pmc_summary.py gpurun_out/NAME profiles/NAME_config5 --tag c5_
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-round}
mkdir -p "$OUT"
B="bench.py"
BT="bench.py --legs none --no-cpu-baseline"   # the headline's kernels alone (the legs run other shapes)
P="bench.py --no-cpu-baseline --parity-chains 0 --steps 5 --warmup 3"
C5="bench.py --no-cpu-baseline --parity-chains 0 --sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --warmup 3 --block-threads 1024"
# the config-5 bench line re-checks its first 4 saved calls of 2 selected chains against the oracle (the CPU
# oracle takes ~25 ms per 1024 x 2048 sweep); the profiled runs skip the parity leg
C5B="${C5/--parity-chains 0/--parity-chains 2 --parity-calls 4}"
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
SQB="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"
if [ "$2" != "skip-tests" ]; then
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit $?
fi
timeout -k 10 500 python $B > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 $BT > "$OUT/prof.log" 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o f -- python3 $P > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o w -- python3 $P > "$OUT/pmc_write.log" 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc $SQA --output-format csv -d "$OUT/pmc_sq" -o s -- python3 $P > "$OUT/pmc_sq.log" 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc $SQB --output-format csv -d "$OUT/pmc_sq_b" -o s -- python3 $P > "$OUT/pmc_sq_b.log" 2>&1 &&
timeout -k 10 200 python $C5B > "$OUT/c5_bench.json" 2> "$OUT/c5_bench.err" &&
timeout -k 10 300 python ${C5B/--warmup 3/--warmup 100} > "$OUT/c5_bench_ss.json" 2> "$OUT/c5_bench_ss.err" && export SR_COOP=0 &&   # (rocprofv3 + cooperative launch: see tools/gpu_c5_round.sh)
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5_prof" -o c5 -- python3 $C5 > "$OUT/c5_prof.log" 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/c5_fetch" -o f -- python3 $C5 > "$OUT/c5_fetch.log" 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/c5_write" -o w -- python3 $C5 > "$OUT/c5_write.log" 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc $SQA --output-format csv -d "$OUT/c5_sq" -o s -- python3 $C5 > "$OUT/c5_sq.log" 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc $SQB --output-format csv -d "$OUT/c5_sq_b" -o s -- python3 $C5 > "$OUT/c5_sq_b.log" 2>&1
rc=$?
echo "exit $rc"
exit $rc
