#!/bin/bash
# kernel time with term kinds removed (SR_EXP 4/8/16 builds): bench ms_per_step each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-exp2}
mkdir -p "$OUT"
for v in full exp4 exp8 exp16 exp1; do
  if [ $v = full ]; then L=seriation-in-paleontological-data-using-mcmc_amd/build/libseriation.so; else L=seriation-in-paleontological-data-using-mcmc_amd/build/$v/libseriation.so; fi
  SERIATION_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 > "$OUT/$v.json" 2>"$OUT/$v.err" || exit 1
  python3 -c "import json;d=json.load(open('$OUT/$v.json'));print('$v', round(d['roofline']['kernel_ms']*1e3/100/100*2400), 'cycles/sweep (2.4GHz est), kernel_ms', round(d['roofline']['kernel_ms'],3))"
done
