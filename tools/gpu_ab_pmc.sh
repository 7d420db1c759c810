#!/bin/bash
# A/B of the current build against build/var/<name> variants (tools/gpu_ab.sh), then the SQ/LDS counter pass
# and an instruction-cache pass on the current build.   tools/gpu_ab_pmc.sh OUTNAME var1 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
bash tools/gpu_ab.sh "$@" || exit 1
B="bench.py --no-cpu-baseline --steps 10 --warmup 10"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d "$OUT/pmc_sq" -o s -- python3 $B > "$OUT/pmc_sq.log" 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH --output-format csv -d "$OUT/pmc_ic" -o i -- python3 $B > "$OUT/pmc_ic.log" 2>&1
echo "icache pass exit $?"
