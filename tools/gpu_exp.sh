#!/bin/bash
# Instruction/cycle counts of the kernel with phases removed (SR_EXP builds), one PMC pass each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-exp}
mkdir -p "$OUT"
B="bench.py --no-cpu-baseline --steps 3 --warmup 1"
for v in full exp1 exp2 exp3; do
  if [ $v = full ]; then L=seriation-in-paleontological-data-using-mcmc_amd/build/libseriation.so; else L=seriation-in-paleontological-data-using-mcmc_amd/build/$v/libseriation.so; fi
  SERIATION_LIB=$L timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$OUT/$v" -o $v -- python3 $B > "$OUT/$v.log" 2>&1 || exit 1
done
