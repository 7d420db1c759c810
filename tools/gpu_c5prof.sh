#!/bin/bash
# Config 5 diagnostics: accepted moves per sweep, the stamp split at TB 1024 and the fine split at
# TB 512 (SR_STAMP_FINE holds <= 8 waves).   tools/gpu_c5prof.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
V=seriation-in-paleontological-data-using-mcmc_amd/build/var
timeout -k 10 200 python tools/acc_probe.py 1024 2048 100 20 > "$OUT/acc_c5.txt" 2>&1 || exit 1
DS=/tmp/sr_synth_1024x2048_20261016.txt
SERIATION_LIB=$V/stamps/libseriation.so timeout -k 10 200 python tools/stamp_profile.py $DS 100 2 1024 > "$OUT/stamps1024.txt" 2>&1 || exit 1
SR_FINE=1 SERIATION_LIB=$V/fine/libseriation.so timeout -k 10 200 python tools/stamp_profile.py $DS 100 2 512 > "$OUT/fine512.txt" 2>&1 || exit 1
cat "$OUT"/*.txt
