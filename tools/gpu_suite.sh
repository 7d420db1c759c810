#!/bin/bash
# The whole GPU check of the current tree: smoke(), the GPU test suite and the default bench line.
#   tools/gpu_suite.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-suite}
mkdir -p "$OUT"
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
tail -3 "$OUT/pytest_gpu.log"
cat "$OUT/bench.json"
echo "exit $rc"
exit $rc
