#!/bin/bash
# New GPU tests, then a PC-sampling profile of the bench (where the sweep kernel's time goes by
# instruction).   tools/gpu_pcsamp.sh OUTNAME [pytest args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
timeout -s KILL 60 rocprofv3 -L > "$OUT/list_avail.txt" 2>&1
grep -i -A12 "pc.sampl" "$OUT/list_avail.txt" | head -40
timeout -s KILL 200 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 50 --output-format csv -d "$OUT/pcs" -o p -- python3 bench.py --no-cpu-baseline --steps 4 --warmup 2 > "$OUT/pcs.log" 2>&1
rc=$?
echo "pc sampling exit $rc"
tail -5 "$OUT/pcs.log"
ls -la "$OUT/pcs"/* 2>/dev/null | head
exit 0
