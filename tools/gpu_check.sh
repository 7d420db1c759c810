#!/bin/bash
# One GPU-box pass: smoke, GPU test suite, bench (with CPU baseline), rocprofv3 kernel stats.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-check}
mkdir -p "$OUT"
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 700 python -m pytest tests -m gpu -x -q -s > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --steps 10 > "$OUT/prof.log" 2>&1
rc=$?
echo "exit $rc"
exit $rc
