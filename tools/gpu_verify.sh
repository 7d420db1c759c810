#!/bin/bash
# Verification pass after a source change: smoke, the whole GPU suite, the default bench line (with its CPU
# baseline and oracle parity leg) and the config-5 line.   tools/gpu_verify.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-verify}
mkdir -p $OUT
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 200 python bench.py --no-cpu-baseline --parity-chains 2 --parity-calls 4 --sites 1024 --taxa 2048 --calls-per-step 2 \
  --steps 20 --warmup 10 --block-threads 1024 > $OUT/c5_bench.json 2> $OUT/c5_bench.err
rc=$?
tail -n 1 $OUT/pytest_gpu.log
echo "exit $rc"
exit $rc
