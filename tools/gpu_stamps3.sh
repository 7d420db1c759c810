#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-st3}
mkdir -p "$OUT"
SERIATION_LIB=seriation-in-paleontological-data-using-mcmc_amd/build/stamps3/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps3.log" 2>&1
rc=$?; sed -e 's/prop draws /draws+cache/; s/terms pi1 /terms     /; s/terms pi2\/swap/barrier wait  /; s/terms pi3 /decide    /; s/decide\/apply\/tail/apply+rest     /' "$OUT/stamps3.log"; exit $rc
