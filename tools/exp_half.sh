set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/half
python3 - <<'PY'
lines = open("tests/golden/datasets/synth_256x512.txt").read().splitlines()
N, M = map(int, lines[0].split())
out = ["%d %d" % (N, 256)]
for l in lines[1:N+1]:
    t = l.split()
    hard = t[-1] == "*"
    vals = t[:M]
    out.append(" ".join(vals[:256]) + (" *" if hard else ""))
open("/tmp/half.txt", "w").write("\n".join(out) + "\n")
PY
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/half/full.json 2>&1 &&
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --dataset /tmp/half.txt > gpurun_out/half/half.json 2>&1 &&
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --dataset /tmp/half.txt --block-threads 512 > gpurun_out/half/half512.json 2>&1
rc=$?
for f in full half half512; do python3 -c "
import json;b=json.load(open('gpurun_out/half/$f.json'));print('$f',b['value'],b['config']['block_threads'],b['roofline']['kernel_ms'])"; done
exit $rc
