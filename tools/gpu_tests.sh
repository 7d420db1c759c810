#!/bin/bash
# Named GPU tests then an optional A/B.   tools/gpu_tests.sh OUTNAME "pytest args" [ab-variant ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; T=$2; shift 2
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest $T -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
if [ $# -gt 0 ]; then bash tools/gpu_ab.sh "$(basename $OUT)_ab" "$@" || exit 1; fi
