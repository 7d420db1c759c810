#!/bin/bash
# (historical recipe: the switches it compares were removed from the kernel source at 289d1cb after this A/B)
# Round-4 config-5 A/B of the word-parallel reversals (seg_reverse_gm) and the prefix rewritten with the
# moved words: the product vs noseg (SR_SEGREV=0: per-bit exchange loop + prefix pass), after the product's
# parity on every HBM-column / split / manycd case.   tools/gpu_ab_r04h.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${1:-r04h}
mkdir -p gpurun_out/${OUT}
timeout -k 10 600 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_edge.py tests/test_gpu_fallbacks.py tests/test_gpu_manycd.py \
  -k "hbm or split or config5 or gm or manycd" -x -q --timeout 150 --timeout-method thread > gpurun_out/${OUT}/parity.log 2>&1 || exit 1
tail -n 1 gpurun_out/${OUT}/parity.log
NOPARITY=1 BENCH_ARGS="--sites 1024 --taxa 2048 --calls-per-step 2 --block-threads 1024" bash tools/gpu_ab.sh ${OUT}_c5 noseg
rc=$?
echo "exit $rc"
exit $rc
