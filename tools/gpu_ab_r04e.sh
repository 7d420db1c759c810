#!/bin/bash
# Round-4 config-5 A/B after reverting to f64 Gibbs checkpoints: the product (f64, one checkpoint per
# word) vs ckg2 (f64, one per word pair: half the scratch stores) vs ck32 (f32, the rejected r04c default);
# parity of the product and ckg2 on the HBM-column / split cases first, then kernel times and the
# fallback counters (tools/c5_fallbacks.py).   tools/gpu_ab_r04e.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${1:-r04e}
V=seriation-in-paleontological-data-using-mcmc_amd/build/var
mkdir -p gpurun_out/${OUT}
timeout -k 10 400 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_edge.py -k "hbm or split or config5" -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/${OUT}/parity_product.log 2>&1 &&
SERIATION_LIB=$V/ckg2/libseriation.so timeout -k 10 400 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_edge.py \
  -k "hbm or split or config5" -x -q --timeout 120 --timeout-method thread > gpurun_out/${OUT}/parity_ckg2.log 2>&1 &&
NOPARITY=1 BENCH_ARGS="--sites 1024 --taxa 2048 --calls-per-step 2 --block-threads 1024" bash tools/gpu_ab.sh ${OUT}_c5 ckg2 ck32 &&
timeout -k 10 120 python tools/c5_fallbacks.py > gpurun_out/${OUT}/fb_product.json &&
SERIATION_LIB=$V/ckg2/libseriation.so timeout -k 10 120 python tools/c5_fallbacks.py > gpurun_out/${OUT}/fb_ckg2.json
rc=$?
echo "exit $rc"
exit $rc
