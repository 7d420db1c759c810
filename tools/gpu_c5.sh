#!/bin/bash
# Config 5 (1024 x 2048, HBM-column variant): parity tests, then timing at two block sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-c5}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_edge.py -x -v --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu-baseline --sites 1024 --taxa 2048 --calls-per-step 2 --steps 3 --warmup 1 --block-threads 512 > "$OUT/bench512.json" 2> "$OUT/bench512.err" &&
timeout -k 10 200 python bench.py --no-cpu-baseline --sites 1024 --taxa 2048 --calls-per-step 2 --steps 3 --warmup 1 --block-threads 1024 > "$OUT/bench1024.json" 2> "$OUT/bench1024.err" &&
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --columns hbm > "$OUT/bench_hbm_256.json" 2> "$OUT/bench_hbm_256.err"
rc=$?
tail -3 "$OUT/pytest.log"; cut -c1-300 "$OUT"/bench*.json
exit $rc
