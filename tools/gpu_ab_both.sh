#!/bin/bash
# A build/var/<name> variant against the product library on one box, interleaved: config 5 (1024 x 2048, split chains,
# 10 warm-up launches of 2 calls) and the headline (256 x 512, 100 chains, the default bench line without legs or CPU
# baseline), each line with its parity leg; then the config-5 and fuzz GPU tests on the variant.
#   tools/gpu_ab_both.sh OUT REPS VARIANT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; REPS=$2; v=$3
mkdir -p "$OUT"
VL=seriation-in-paleontological-data-using-mcmc_amd/build/var/$v/libseriation.so
C5="--no-cpu-baseline --legs none --sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --warmup 10 --parity-chains 2 --parity-rejected 0 --parity-calls 4"
C3="--no-cpu-baseline --legs none"
show() { python3 -c "import json;b=json.load(open('$1'));print('$2', round(b['roofline']['kernel_ms'],3), round(b['value']), b['parity']['match'])"; }
for rep in $(seq 1 $REPS); do
  timeout -k 10 200 python bench.py $C5 > "$OUT/c5_product_$rep.json" 2> "$OUT/c5_product_$rep.err" && show "$OUT/c5_product_$rep.json" "c5 product $rep" &&
  SERIATION_LIB=$VL timeout -k 10 200 python bench.py $C5 > "$OUT/c5_${v}_$rep.json" 2> "$OUT/c5_${v}_$rep.err" && show "$OUT/c5_${v}_$rep.json" "c5 $v $rep" &&
  timeout -k 10 200 python bench.py $C3 > "$OUT/c3_product_$rep.json" 2> "$OUT/c3_product_$rep.err" && show "$OUT/c3_product_$rep.json" "c3 product $rep" &&
  SERIATION_LIB=$VL timeout -k 10 200 python bench.py $C3 > "$OUT/c3_${v}_$rep.json" 2> "$OUT/c3_${v}_$rep.err" && show "$OUT/c3_${v}_$rep.json" "c3 $v $rep" || exit 1
done
[ -n "$NO_TESTS" ] && exit 0
SERIATION_LIB=$VL timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_config5.py tests/test_gpu_fuzz.py > "$OUT/pytest_$v.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_$v.log"
exit $rc
