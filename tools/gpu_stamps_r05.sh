#!/bin/bash
# Phase stamps of config 3 (coarse and fine stamp builds of the current source) and one bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05g}
mkdir -p "$OUT"
V=$PWD/seriation-in-paleontological-data-using-mcmc_amd/build/var
SERIATION_LIB=$V/stamps/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps.txt" 2>&1 &&
SR_FINE=1 SERIATION_LIB=$V/fine/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps_fine.txt" 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
cat "$OUT/stamps.txt" "$OUT/stamps_fine.txt"
echo "exit $rc"
exit $rc
