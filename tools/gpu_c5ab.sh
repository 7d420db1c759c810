#!/bin/bash
# Config 5 (1024 x 2048, split chains) A/B: config 5 + forced-exact GPU tests and the parity subset on the
# default library, then tools/gpu_ab.sh with the config-5 bench arguments against build/var/<VARS>.
#   OUTN=r03z_c5 VARS="name ..." tools/gpu_c5ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/${OUTN:-r03z_c5}
timeout -k 10 400 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_fallbacks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${OUTN:-r03z_c5}/tests.log 2>&1 || { tail -30 gpurun_out/${OUTN:-r03z_c5}/tests.log; exit 1; }
tail -1 gpurun_out/${OUTN:-r03z_c5}/tests.log
BENCH_ARGS="--sites 1024 --taxa 2048 --calls-per-step 2 --block-threads 1024" bash tools/gpu_ab.sh ${OUTN:-r03z_c5}ab ${VARS:-c5old}
