#!/bin/bash
# Round 5: phase split and phase-C batch statistics at a chain's steady state (stamp builds, after 500 warm-up
# calls: the bench's timed region starts after 500) next to the fresh-chain split.   tools/gpu_r05s.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05s}
mkdir -p "$OUT"
V=$PWD/seriation-in-paleontological-data-using-mcmc_amd/build/var
SR_WARM=500 SERIATION_LIB=$V/stamps/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps_warm.txt" 2>&1 &&
SR_WARM=500 SR_FINE=1 SERIATION_LIB=$V/fine/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps_fine_warm.txt" 2>&1 &&
SR_WARM=1500 SERIATION_LIB=$V/stamps/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps_warm1500.txt" 2>&1
rc=$?
cat "$OUT"/stamps_*.txt
exit $rc
