#!/bin/bash
# Round 6, first box pass: the new GPU tests (certification self-tests + negative control, fixed-seed fuzz, the
# ragged three-rank bench rehearsal, checkpoints with their record capacity), the default bench line with its
# config2 / config5 legs, then the planner A/B for mid-size shapes (341 x 890 and two more: 512-thread LDS
# columns against 1024-thread HBM columns, interleaved).  Each GPU step has its own limit; the chain stops at the
# first failure.    tools/gpu_r06a.sh NAME
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06a}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_cert.py tests/test_gpu_fuzz.py tests/test_gpu_rccl.py \
  tests/test_gpu_edge.py::test_checkpoint_carries_records tests/test_cli.py} -m gpu -x -v --timeout 400 \
  --timeout-method thread > "$OUT/pytest_new.log" 2>&1 || { tail -40 "$OUT/pytest_new.log"; exit 1; }
tail -3 "$OUT/pytest_new.log"
timeout -k 10 300 python tests/cert_run.py > "$OUT/cert_product.json" 2> "$OUT/cert.err" &&
SERIATION_LIB=seriation-in-paleontological-data-using-mcmc_amd/build/cert8/libseriation.so \
  timeout -k 10 300 python tests/cert_run.py > "$OUT/cert_shift8.json" 2>> "$OUT/cert.err" || exit 1
timeout -k 10 500 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python3 tools/ab_planner.py "$OUT" || exit 1
echo done
