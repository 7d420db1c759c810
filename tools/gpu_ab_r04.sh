#!/bin/bash
# Round-4 same-box A/Bs: config 3 (256 x 512, the bench) default vs the kernarg-reload variant; config 5
# (1024 x 2048, split chains) default (f32 Gibbs checkpoints per word) vs f64 checkpoints (ck64) and f32
# checkpoints per word pair (ckg2).  Variants are
# built here by tools/build_variant.sh (self-contained: own snapshot and spec defines).
#   tools/gpu_ab_r04.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${1:-r04ab}
V=seriation-in-paleontological-data-using-mcmc_amd/build/var
mkdir -p gpurun_out/${OUT}_parity
# each variant's parity first (the HBM-column / split cases for the checkpoint variants, the bench shape for karg)
SERIATION_LIB=$V/karg/libseriation.so timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q \
  > gpurun_out/${OUT}_parity/karg.log 2>&1 &&
SERIATION_LIB=$V/ckg2/libseriation.so timeout -k 10 400 python -m pytest tests/test_gpu_config5.py tests/test_gpu_edge.py \
  -k "hbm or split or config5" -x -q > gpurun_out/${OUT}_parity/ckg2.log 2>&1 &&
NOPARITY=1 bash tools/gpu_ab.sh ${OUT}_karg karg &&
NOPARITY=1 BENCH_ARGS="--sites 1024 --taxa 2048 --calls-per-step 2 --block-threads 1024" bash tools/gpu_ab.sh ${OUT}_c5 ck64 ckg2
rc=$?
echo "exit $rc"
exit $rc
