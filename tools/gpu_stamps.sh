#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-st}
mkdir -p "$OUT"
SERIATION_LIB=seriation-in-paleontological-data-using-mcmc_amd/build/stamps/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps.log" 2>&1
rc=$?; cat "$OUT/stamps.log"; exit $rc
