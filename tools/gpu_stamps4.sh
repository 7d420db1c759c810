#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-st4}
mkdir -p "$OUT"
SR_GIBBS_STATS=1 SERIATION_LIB=seriation-in-paleontological-data-using-mcmc_amd/build/stamps4/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps4.log" 2>&1
rc=$?; sed -e 's/totals+c,d /A totals   /; s/sampleab   /B pass0+pre/; s/logl /B p1 /; s/prop draws /B pass2    /; s/terms pi1 /B tail    /; s/terms pi2\/swap/A draws+setup /; s/terms pi3 /phase C   /; s/decide\/apply\/tail/C rest+tail     /' "$OUT/stamps4.log"; exit $rc
