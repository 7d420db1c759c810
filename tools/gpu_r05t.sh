#!/bin/bash
# Round 5: coarse stamps at steady state with the phase-C counters (batches, proposals drawn, table refills,
# scalar-path proposals).   tools/gpu_r05t.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05t}
mkdir -p "$OUT"
V=$PWD/seriation-in-paleontological-data-using-mcmc_amd/build/var
SR_WARM=500 SERIATION_LIB=$V/stamps/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps_warm.txt" 2>&1
rc=$?
cat "$OUT"/stamps_*.txt
exit $rc
