#!/bin/bash
# (historical recipe: the switches it compares were removed from the kernel source at 289d1cb after this A/B)
# Round-4 config-5 A/B of the split kernel's register-resident own-taxon state (SR_APREG), tagged exchanges
# (SR_XTAG) and fused Gibbs passes 0/1 (SR_FUSE01): product vs apreg, xtag, xtap (both), fuse, fuap (fuse +
# apreg); parity of fuap, fuse and xtap on the HBM-column / split cases first.   tools/gpu_ab_r04j.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${1:-r04j}
V=seriation-in-paleontological-data-using-mcmc_amd/build/var
mkdir -p gpurun_out/${OUT}
for v in fuap fuse xtap; do
  SERIATION_LIB=$V/$v/libseriation.so timeout -k 10 400 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_edge.py \
    tests/test_gpu_fallbacks.py -k "hbm or split or config5" -x -q --timeout 150 --timeout-method thread > gpurun_out/${OUT}/parity_$v.log 2>&1 || exit 1
  tail -n 1 gpurun_out/${OUT}/parity_$v.log
done
NOPARITY=1 BENCH_ARGS="--sites 1024 --taxa 2048 --calls-per-step 2 --block-threads 1024" bash tools/gpu_ab.sh ${OUT}_c5 apreg xtag xtap fuse fuap
rc=$?
[ $rc -eq 0 ] && SERIATION_LIB=$V/fuap/libseriation.so timeout -k 10 120 python tools/c5_fallbacks.py > gpurun_out/${OUT}/fb_fuap.json
rc=$?
echo "exit $rc"
exit $rc
