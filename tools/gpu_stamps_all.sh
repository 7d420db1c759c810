#!/bin/bash
# Phase stamps of the sweep kernel (SR_STAMPS builds): default split, Gibbs split, draws split, decide split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-stamps}
mkdir -p "$OUT"
B=seriation-in-paleontological-data-using-mcmc_amd/build
SERIATION_LIB=$B/stamps/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps.log" 2>&1 &&
SERIATION_LIB=$B/stamps4/libseriation.so SR_GIBBS_STATS=1 timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps_gibbs.log" 2>&1 &&
SERIATION_LIB=$B/stamps3/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps_decide.log" 2>&1 &&
SERIATION_LIB=$B/stamps2/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps_draws.log" 2>&1
rc=$?
cat "$OUT"/stamps*.log
exit $rc
