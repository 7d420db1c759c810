#!/bin/bash
# Round 5: A/B of two-words-ahead Gibbs byte-table reads (SR_GIBBS_AHEAD=2) with parity, then the coarse stamp
# build's phase split with the phase-C batch statistics.   tools/gpu_r05r.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${1:-r05r}
V=$PWD/seriation-in-paleontological-data-using-mcmc_amd/build/var
bash tools/gpu_ab_par.sh "$OUT" ahead2 || exit 1
SERIATION_LIB=$V/stamps/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "gpurun_out/$OUT/stamps.txt" 2>&1
rc=$?
cat "gpurun_out/$OUT/stamps.txt"
exit $rc
