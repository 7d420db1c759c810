#!/bin/bash
# Round-4 config-5 A/B of the grouped Gibbs checkpoints (f64, one per SR_CKG window words): the product
# (SR_CKG=2) vs ckg4 vs ckg1 (r03's one per word); parity of the product and ckg4 on the HBM-column /
# split cases first; then the split kernel's phase stamps (build/var/stamps).   tools/gpu_ab_r04f.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${1:-r04f}
V=seriation-in-paleontological-data-using-mcmc_amd/build/var
mkdir -p gpurun_out/${OUT}
for lib in product ckg4; do
  L=""; [ $lib = product ] || L=$V/$lib/libseriation.so
  SERIATION_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_edge.py tests/test_gpu_fallbacks.py \
    -k "hbm or split or config5" -x -q --timeout 120 --timeout-method thread > gpurun_out/${OUT}/parity_$lib.log 2>&1 || exit 1
done
NOPARITY=1 BENCH_ARGS="--sites 1024 --taxa 2048 --calls-per-step 2 --block-threads 1024" bash tools/gpu_ab.sh ${OUT}_c5 ckg4 ckg1 || exit 1
python tools/gen_synthetic.py 1024 2048 20261016 /tmp/sr_synth_1024x2048_20261016.txt &&
SERIATION_LIB=$V/stamps/libseriation.so timeout -k 10 200 python tools/stamp_profile.py /tmp/sr_synth_1024x2048_20261016.txt 100 2 1024 \
  > gpurun_out/${OUT}/stamps_c5.txt 2>&1
rc=$?
echo "exit $rc"
exit $rc
