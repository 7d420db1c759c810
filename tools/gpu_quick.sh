#!/bin/bash
# Quick GPU iteration: parity tests, phase stamps, short bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}
mkdir -p "$OUT"
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_e2e.py -k "not config2 and not launcher" -x -q > "$OUT/parity.log" 2>&1 &&
SERIATION_LIB=seriation-in-paleontological-data-using-mcmc_amd/build/stamps/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > "$OUT/stamps.log" 2>&1 &&
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
tail -2 "$OUT/parity.log"; cat "$OUT/stamps.log" "$OUT/bench.json" 2>/dev/null | cut -c1-400
exit $rc
