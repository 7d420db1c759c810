#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-st2}
mkdir -p "$OUT"
SERIATION_LIB=seriation-in-paleontological-data-using-mcmc_amd/build/stamps2/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps2.log" 2>&1
rc=$?; sed -e 's/prop draws /batch setup/; s/terms pi1 /draw loop /; s/terms pi2\/swap/taxon cache   /; s/terms pi3 /terms all /' "$OUT/stamps2.log"; exit $rc
