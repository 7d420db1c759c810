#!/bin/bash
# Round 5, first pass: smoke, the GPU suite, the default bench line, then the phase stamps of config 3
# (coarse and fine stamp builds, tools/build_variant.sh stamps / fine) for the phase-C work.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05a}
mkdir -p "$OUT"
V=seriation-in-paleontological-data-using-mcmc_amd/build/var
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
SERIATION_LIB=$PWD/$V/stamps/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps.txt" 2>&1 &&
SR_FINE=1 SERIATION_LIB=$PWD/$V/fine/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps_fine.txt" 2>&1
rc=$?
echo "exit $rc"
exit $rc
