set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03z_c5
timeout -k 10 400 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_fallbacks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03z_c5/tests.log 2>&1 || { tail -30 gpurun_out/r03z_c5/tests.log; exit 1; }
tail -1 gpurun_out/r03z_c5/tests.log
BENCH_ARGS="--sites 1024 --taxa 2048 --calls-per-step 2 --block-threads 1024" bash tools/gpu_ab.sh r03z_c5ab c5old
