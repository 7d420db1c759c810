#!/bin/bash
# Config 5 (1024 x 2048, split chains): the product library against build/var/<name> variants, interleaved on one box
# at a fixed chain age (WARM warm-up launches of 2 calls, default 10 as profiles/r05n), each line with its parity leg
# (2 selected chains x 4 saved calls against the oracle).     tools/gpu_c5_variants.sh OUT REPS var...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; REPS=$2; shift 2
mkdir -p "$OUT"
V=seriation-in-paleontological-data-using-mcmc_amd/build/var
C5="--no-cpu-baseline --legs none --sites 1024 --taxa 2048 --calls-per-step 2 --steps 10 --warmup ${WARM:-10} --parity-chains 2 --parity-rejected 0 --parity-calls 4"
for rep in $(seq 1 $REPS); do
  timeout -k 10 200 python bench.py $C5 > "$OUT/product_$rep.json" 2> "$OUT/product_$rep.err" || exit 1
  echo "product $rep $(python3 -c "import json;b=json.load(open('$OUT/product_$rep.json'));print(round(b['roofline']['kernel_ms'],3), b['parity']['match'])")"
  for v in "$@"; do
    SERIATION_LIB=$V/$v/libseriation.so timeout -k 10 200 python bench.py $C5 > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || exit 1
    echo "$v $rep $(python3 -c "import json;b=json.load(open('$OUT/${v}_$rep.json'));print(round(b['roofline']['kernel_ms'],3), b['parity']['match'])")"
  done
done
