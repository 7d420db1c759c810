#!/bin/bash
# Config 5 phase split of the split kernel (SR_STAMPS builds: coarse, and SR_STAMP_DECIDE's split of phase C:
# 3 draws+cache, 4 terms, 5 exchange/barrier, 6 decide+scan, 7 apply+rest), after the product's parity on
# the HBM-column / split cases.   tools/gpu_c5_stamps_r04.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04g}
V=seriation-in-paleontological-data-using-mcmc_amd/build/var
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_edge.py tests/test_gpu_fallbacks.py \
  -k "hbm or split or config5" -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1 || exit 1
python tools/gen_synthetic.py 1024 2048 20261016 /tmp/sr_synth_1024x2048_20261016.txt || exit 1
for v in stamps stamps3; do
  SERIATION_LIB=$V/$v/libseriation.so timeout -k 10 200 python tools/stamp_profile.py /tmp/sr_synth_1024x2048_20261016.txt 100 2 1024 \
    > $OUT/c5_$v.txt 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --parity-chains 0 --steps 20 --warmup 10 --sites 1024 --taxa 2048 \
  --calls-per-step 2 --block-threads 1024 > $OUT/c5_bench.json 2> $OUT/c5_bench.err
rc=$?
echo "exit $rc"
exit $rc
