#!/bin/bash
# Config 5: the product against one build/var/<name> variant of the split kernels (interleaved, tools/gpu_c5_variants.sh),
# then the GPU tests that run HBM-column / split kernels, on the variant.
#   tools/gpu_c5_ab_tests.sh OUT REPS VARIANT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=$1; REPS=$2; v=$3
bash tools/gpu_c5_variants.sh "$OUT" "$REPS" "$v" || exit $?
SERIATION_LIB=seriation-in-paleontological-data-using-mcmc_amd/build/var/$v/libseriation.so timeout -k 10 700 \
  python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_config5.py tests/test_gpu_fuzz.py \
  tests/test_gpu_edge.py tests/test_gpu_multi.py tests/test_gpu_philox.py ${EXTRA_TESTS:-} > "gpurun_out/$OUT/pytest_$v.log" 2>&1; rc=$?
tail -3 "gpurun_out/$OUT/pytest_$v.log"
exit $rc
