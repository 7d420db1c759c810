#!/usr/bin/env python3
"""Benchmark: chain-iterations/s of the MCMC seriation sweep on MI355X.

Headline (BASELINE.json metric, configs[2]): synthetic 256 sites x 512 taxa (tools/gen_synthetic.py,
seed 20261015), 100 chains in total, sharded contiguously over the N GPUs (ragged shards from
dist.shard: 13/13/13/13/12/12/12/12 at N = 8; `--total-chains 800` is config 4, `--chains-per-gpu C`
the weak-scaling form).  One step = one kernel launch that runs `--calls-per-step` reference
mcmc_sample calls (10 sweeps each, mcmc.c:225) for every chain of the rank and saves one record per
call (a, b, pi, c, d, loglik -- the mcmc_save_chain payload) to HBM, as the reference's sampling phase
does.  Chain state, dataset and records stay resident in HBM; host formatting of records is not timed.
At the end of the timed region ranks all-gather their per-chain summaries over RCCL (the one-sigma
selection input) and the selected chains' records -- the only collectives.

At N = 1 the same line also carries (`--legs`, default both):
  config2 -- the reference's own published workload (Report p.6 s5.1: g10s10, 100 chains x 2000
             mcmc_sample calls in 15-20 min): script.py:48-67 end to end through the drop-in launcher,
             Chains/chain_NN files written, beside the CPU oracle CLI running the same protocol, whose
             files must be byte-identical;
  config5 -- 1024 x 2048 (HBM columns, split chains), 100 chains from init over the reference protocol
             (1000 burn-in + 1000 saved calls), with the steady-state rate of the saved window and its
             records checked against the committed oracle digests (tests/golden/config5.json).

1 chain-iteration = 1 sweep = body of mcmc.c:225-244.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

SYNTH = os.path.join(ROOT, "tests", "golden", "datasets", "synth_256x512.txt")
G10S10 = os.path.join(ROOT, "tests", "golden", "datasets", "g10s10.txt")
C5_GOLDEN = os.path.join(ROOT, "tests", "golden", "config5.json")
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
CHAINS_SELECTED = 8    # choose_chains(8) as in Report Table 1 for g10s10


def launch_ranks(n):
    """python bench.py --gpus N without a launcher: start N ranks with torch.distributed.run
    (one process per GPU, rendezvous on 127.0.0.1) as a child process and return its status."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def visible_gpu_count(base="/sys/class/kfd/kfd/topology/nodes"):
    """GPUs this process could use, counted without initialising HIP (torch.cuda.device_count() may fall back to
    hipGetDeviceCount, and this process must not touch the GPU before it starts the ranks): the KFD topology's
    nodes with SIMDs, narrowed by ROCR / HIP / CUDA_VISIBLE_DEVICES.  None when the topology cannot be read
    (then the ranks report a missing device themselves)."""
    try:
        nodes = os.listdir(base)
    except OSError:
        return None
    n = 0
    for node in nodes:
        try:
            with open(os.path.join(base, node, "properties")) as fh:
                for line in fh:
                    k, _, v = line.partition(" ")
                    if k == "simd_count" and int(v) > 0:
                        n += 1
                        break
        except (OSError, ValueError):
            return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None and v.strip():
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def algorithmic_bytes_per_iter(N, M):
    """B_iter = N*M (one pass over X for the Gibbs a/b update) + 48*M
    (a, b, t0, f0, t1, f1 read+write) + 16*9*M (16 proposals x (a, b + one row/column slice))."""
    return N * M + 192 * M


def measured_traffic(N, M, chains, sweeps_per_step):
    """HBM bytes per sweep-kernel launch from the latest round's PMC summary in profiles/ whose workload
    matches (tools/pmc_summary.py: 2*FETCH_SIZE + WRITE_SIZE from separate rocprofv3 --pmc passes
    over this bench; rounds are ordered by file name, r01c < ... < r02g, not by mtime, which a checkout
    or a copy to the GPU box does not keep).  None when no matching PMC pass exists."""
    import glob
    best = None
    for p in glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")):
        try:
            with open(p) as fh:
                t = json.load(fh)
            w = t.get("workload") or {}
            if (w.get("sites"), w.get("taxa"), w.get("chains_per_gpu"), w.get("sweeps_per_step")) != \
                    (N, M, chains, sweeps_per_step) or "traffic_bytes_per_launch" not in t:
                continue
            if best is None or os.path.basename(p) > best[0]:
                best = (os.path.basename(p), p, t)
        except (OSError, ValueError):
            continue
    if best is None:
        return None, None, {}
    return best[2]["traffic_bytes_per_launch"], os.path.relpath(best[1], ROOT), best[2]


def _cpu_worker(args):
    text, seed, burnin, calls, variant = args
    import oracle_ref
    if variant != "O2":
        oracle_ref.use_variant(variant)
    o = oracle_ref.run_chain(text, seed, burnin, calls, sweeps=10)
    return o["burnin_s"], o["sample_s"], o["rc"]


def cpu_share():
    """CPU cores this process may use: the launcher's thread budget (OMP_NUM_THREADS: the GPU
    box's per-GPU share; its nproc counts the whole machine), else the affinity mask and the
    cgroup quota."""
    nproc = os.cpu_count() or 1
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n, nproc


def cpu_baseline(path, burnin, calls, workers, variant="O2"):
    """The CPU oracle (C restatement of mcmc.c; recount after every accepted proposal as the reference) on
    `workers` processes, one chain each: `burnin` untimed mcmc_sample calls from chain birth -- the calls the
    GPU's warm-up runs, so both sides time chains of the same age (mcmc.c:140-185) -- then `calls` timed calls.
    value = the sum of the workers' rates over the timed window (one chain per core); "from_birth" = the same
    over the burn-in window (young chains accept far more moves, each paid with an O(N*M) recount).
    variant "O2" (gcc -O2) or "O0" (reference-like: the shipped binary was built at -O0)."""
    import multiprocessing as mp
    with open(path, "rb") as fh:
        text = fh.read()
    import oracle_ref
    oracle_ref.lib()  # build/load before forking
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    pool = ctx.Pool(workers)
    try:
        res = pool.map(_cpu_worker, [(text, s + 1, burnin, calls, variant) for s in range(workers)])
    finally:
        # close + join: the workers exit on their own (a Pool context exit terminate()s them with
        # SIGTERM, which a profiler's signal handler reports as an abort)
        pool.close()
        pool.join()
    wall = time.perf_counter() - t0
    assert all(rc == 0 for _, _, rc in res)
    share, nproc = cpu_share()
    value = sum(calls * 10 / ts for _, ts, _ in res)
    out = {"value": value, "unit": "chain-iterations/s", "cores": workers, "kind": "port",
           "nproc": nproc, "cpu_share": share,
           "sample": "%d chains, each %d untimed mcmc_sample calls from birth (the GPU's warm-up calls) then %d timed "
                     "calls (%d sweeps each) of the bench workload; oracle/ (C restatement of mcmc.c, gcc -%s, recount "
                     "after accept as the reference) on %d processes (one per core of this process's CPU share; nproc "
                     "%d); value = sum of the per-chain rates over the timed window; wall %.1f s"
                     % (workers, burnin, calls, 10, variant, workers, nproc, wall)}
    if burnin:
        out["from_birth"] = {"value": sum(burnin * 10 / tb for tb, _, _ in res), "unit": "chain-iterations/s",
                             "sample": "the same chains over their first %d calls (from birth: the regime a fresh "
                                       "chain runs in, not the GPU's timed window)" % burnin}
    return out


def leg_config2_cpu(workers, tmp):
    """config2's CPU side, before the GPU is touched: the oracle CLI (oracle/build/mcmc_oracle, the reference
    main() restated, mcmc.c:102-210) as script.py:25-45 starts it -- `mcmc k` with GSL_RNG_SEED = k + 1 in its own
    directory -- for chains 0..workers-1 of the 100, one process per core, full protocol (1000 burn-in + 1000 saved
    calls), files written.  Their Chains/ files are the parity reference of the GPU run."""
    import subprocess
    cli = os.path.join(ROOT, "oracle", "build", "mcmc_oracle")
    if not os.path.exists(cli):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    procs = []
    t0 = time.perf_counter()
    for k in range(workers):
        d = os.path.join(tmp, "cpu%02d" % k)
        os.makedirs(os.path.join(d, "Chains", "chain_%02d" % k))
        with open(G10S10, "rb") as fin:
            procs.append(subprocess.Popen([cli, str(k)], cwd=d, stdin=fin, stdout=subprocess.DEVNULL,
                                          stderr=subprocess.DEVNULL, env=dict(os.environ, GSL_RNG_SEED=str(k + 1))))
    rcs = [p.wait() for p in procs]
    wall = time.perf_counter() - t0
    assert all(rc == 0 for rc in rcs), rcs
    rate = workers * 2000 * 10 / wall
    return {"chains": workers, "cores": workers, "wall_s": wall, "chain_iterations_per_s": rate,
            "projected_100_chain_wall_s": 100 * 2000 * 10 / rate, "kind": "port (oracle CLI, gcc -O2)",
            "sample": "chains 0..%d of the 100 (seeds 1..%d), the full protocol each, one process per core, files "
                      "written; 100-chain wall projected at the same rate" % (workers - 1, workers)}


def leg_config2_gpu(device, tmp, cpu):
    """config2 on the GPU: launcher.run_all_chains (script.py:48-67) over g10s10 with seeds 1..100 -- dataset load,
    init, 1000 burn-in + 1000 saved calls per chain, the five Chains/chain_NN files per chain, the closing
    mcmc_consistent -- timed end to end; then the files of the chains the CPU ran compared byte for byte."""
    from seriation_amd import launcher
    root = os.path.join(tmp, "gpu")
    t0 = time.perf_counter()
    summ = launcher.run_all_chains(G10S10, n_chains=100, seeds=list(range(1, 101)), devices=[device], root=root,
                                   verbose=False)
    wall = time.perf_counter() - t0
    files = ("chain_data.csv", "exp_data.csv", "taxa.csv", "sites.csv", "hard_sites.csv")
    bad = []
    nchk = cpu["chains"] if cpu else 0
    for k in range(nchk):
        for f in files:
            with open(os.path.join(tmp, "cpu%02d" % k, "Chains", "chain_%02d" % k, f), "rb") as fa, \
                    open(os.path.join(root, "Chains", "chain_%02d" % k, f), "rb") as fb:
                if fa.read() != fb.read():
                    bad.append("chain_%02d/%s" % (k, f))
    out = {"workload": "Dataset/g10s10.txt (124 sites x 139 taxa), 100 chains (seeds 1..100), 1000 burn-in + 1000 "
                       "saved mcmc_sample calls each (script.py:48-67 -> mcmc.c:102-210), Chains/chain_NN/*.csv written",
           "gpu_wall_s": wall, "chain_iterations_per_s": 100 * 2000 * 10 / wall,
           "consistent": all(s["consistent"] == 0 for s in summ),
           "timed": "launcher.run_all_chains end to end: Dataset.load, init, sampling, file output, closing "
                    "mcmc_consistent",
           "reference_published": {"wall_s": [900, 1200], "source": "Docs/Report.pdf p.6 s5.1: 100 chains x 2000 "
                                   "mcmc_sample calls in 15-20 min (6 processes)"},
           "speedup_vs_published": [900 / wall, 1200 / wall],
           "cpu": cpu}
    if cpu:
        out["parity"] = {"chains": list(range(nchk)), "files": list(files), "match": not bad, "mismatch": bad,
                         "note": "the GPU run's Chains/chain_NN files byte-identical to the oracle CLI's"}
        out["speedup_vs_cpu_oracle"] = cpu["projected_100_chain_wall_s"] / wall
    return out


def leg_config5(device, calls_per_launch=50):
    """config5 (BASELINE configs[4]): synthetic 1024 x 2048 (gen_synthetic seed 20261016), 100 chains (seeds
    1..100) from init over the reference protocol, 1000 burn-in + 1000 saved calls (mcmc.c:140-185), launches of
    `calls_per_launch` calls.  Timed: the whole protocol from session creation (host init, upload) to the last
    record, and the saved window alone (the steady-state rate).  Parity: chains 0..3 against the committed
    oracle digests of tests/golden/config5.json (every saved record, exp_data)."""
    import hashlib as hl
    import numpy as np
    import gen_synthetic
    import seriation_amd as sa
    X, hard = gen_synthetic.make(1024, 2048, 20261016)
    text = gen_synthetic.to_text(X, hard).encode()
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = list(range(1, 101))
    launches = 1000 // calls_per_launch
    t0 = time.perf_counter()
    sess = sa.Session(ds, seeds, device=device, calls_per_launch=1000)
    t_created = time.perf_counter()
    for _ in range(launches):
        sess.run(calls_per_launch, save=False)
    sess.sync()
    t1 = time.perf_counter()
    for _ in range(launches):
        sess.run(calls_per_launch, save=True)
    sess.sync()
    t2 = time.perf_counter()
    rows = sess.summaries()
    t3 = time.perf_counter()
    kernel, variant = sess.kernel, sess.variant
    launch = ("ordinary (SR_COOP=0)" if os.environ.get("SR_COOP") == "0" else "cooperative") if kernel == "split" \
        else "ordinary"
    parity = None
    if os.path.exists(C5_GOLDEN):
        with open(C5_GOLDEN) as fh:
            g = json.load(fh)
        bad = {}
        if g["dataset_sha256"] != hl.sha256(text).hexdigest():
            bad["dataset"] = "generated matrix differs from the fixture's"
        for ch in g["chains"]:
            k = ch["seed"] - 1
            ab, cd = sess.fetch_chain_records(k)
            dig = [hl.sha256(np.ascontiguousarray(r, dtype="<i4").tobytes()).hexdigest() for r in ab]
            n = len(ch["sha256"])
            if dig[:n] != ch["sha256"]:
                bad[str(k)] = "integer state differs from saved call %d on" % next(
                    i for i in range(n) if dig[i] != ch["sha256"][i])
            elif [[float(v).hex() for v in r] for r in cd[:n]] != ch["cdl_hex"]:
                bad[str(k)] = "c/d/loglik bits differ"
            elif [float(v).hex() for v in rows[k, 1:4]] != ch["exp_hex"]:
                bad[str(k)] = "exp_data differs"
        parity = {"chains": [ch["seed"] - 1 for ch in g["chains"]], "seeds": [ch["seed"] for ch in g["chains"]],
                  "burnin_calls": g["burnin_calls"], "saved_calls_compared": g["saved_calls"], "match": not bad,
                  "mismatch": bad, "reference": "tests/golden/config5.json (oracle/om_mcmc.c digests, "
                                                "tests/golden/make_golden_c5.py)"}
    sess.close()
    iters = 100 * 2000 * 10
    return {"workload": "synthetic (tools/gen_synthetic.py seed 20261016) 1024 sites x 2048 taxa, 12 hard sites, 100 "
                        "chains (seeds 1..100) from init, 1000 burn-in + 1000 saved mcmc_sample calls, %d-call launches"
                        % calls_per_launch,
            "columns": variant, "kernel": kernel, "launch": launch,
            "protocol_wall_s": t3 - t0, "protocol_chain_iterations_per_s": iters / (t3 - t0),
            "session_create_s": t_created - t0, "burnin_wall_s": t1 - t_created, "saved_window_wall_s": t2 - t1,
            "steady_state_chain_iterations_per_s": iters / 2 / (t2 - t1),
            "timed": "protocol: session creation (the chains' host initialisation on the CPU share's threads + upload) "
                     "to the exp_data summaries; steady state: the 1000 saved calls (10 000 sweeps per chain after "
                     "10 000 of burn-in)",
            "parity": parity}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=20, help="untimed steps first (the clocks ramp over the first ~10 launches)")
    ap.add_argument("--total-chains", type=int, default=100, help="chains in the whole job, sharded contiguously over "
                    "the N GPUs (ragged shards: dist.shard); the metric's 100 at every N (strong scaling); 800 = config 4")
    ap.add_argument("--chains-per-gpu", type=int, default=0, help="weak scaling instead: this many chains per GPU "
                    "(overrides --total-chains)")
    ap.add_argument("--calls-per-step", type=int, default=50,
                    help="mcmc_sample calls per step: 50 (500 sweeps) makes the driver's --steps 20 --warmup 5 time "
                         "SURVEY 8(d)'s 10 000 sweeps after 2 500 warm-up sweeps, saving 1000 records per chain")
    ap.add_argument("--dataset", default=SYNTH)
    ap.add_argument("--sites", type=int, default=0, help="synthetic N x M instead of --dataset "
                    "(seed 20261015 for 256x512, 20261016 otherwise: SURVEY.md 8(d) configs 3 and 5)")
    ap.add_argument("--taxa", type=int, default=0)
    ap.add_argument("--columns", default="auto", choices=("auto", "lds", "hbm"))
    ap.add_argument("--cpu-calls", type=int, default=600)
    ap.add_argument("--cpu-workers", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--block-threads", type=int, default=0)
    ap.add_argument("--rng", default="mt", choices=("mt", "philox"), help="philox: the opt-in counter-based stream "
                    "(SR_F_RNG_PHILOX; not the reference's, so never the headline line)")
    ap.add_argument("--generic", action="store_true", help="the generic kernel (shape from the launch "
                    "arguments) instead of the default one compiled for the dataset's shape (SR_F_GENERIC_KERNEL)")
    ap.add_argument("--parity-chains", type=int, default=CHAINS_SELECTED, help="after the timed region, rerun this many "
                    "of the selected chains plus --parity-rejected chains the selection rejected on the CPU oracle "
                    "(burn-in = the warm-up calls) and require every compared saved record of the timed region to match "
                    "bit for bit (0: skip)")
    ap.add_argument("--parity-rejected", type=int, default=2, help="chains the one-sigma selection rejected that the "
                    "parity leg also checks (the first and the last of rank 0's shard that were not selected)")
    ap.add_argument("--parity-calls", type=int, default=-1, help="compare only the first K saved records of each "
                    "checked chain (0: all; -1 auto: all for LDS-column sessions, 4 for HBM columns, whose oracle "
                    "takes ~0.4 s per call)")
    ap.add_argument("--device-of-rank", default="", help="comma-separated HIP ordinal per local rank (default: the "
                    "local rank), e.g. 0,0 to rehearse two ranks on one GPU")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"), help="torch.distributed backend under "
                    "a launcher: nccl = RCCL over xGMI (one rank per GPU); gloo = host collectives (rehearsals with "
                    "several ranks on one GPU, which RCCL does not allow)")
    ap.add_argument("--no-save", action="store_true", help="sample without saving records (SURVEY.md 8(d) "
                    "asks for both; the default saves one record per call, as the reference's sampling phase)")
    ap.add_argument("--legs", default="auto", help="extra workloads in the same line at N = 1 (ignored at N > 1): "
                    "comma-separated from config2, config5; none; auto = both unless --no-cpu-baseline or N > 1")
    args = ap.parse_args()
    legs = set()
    if args.legs == "auto":
        if args.gpus == 1 and not args.no_cpu_baseline:
            legs = {"config2", "config5"}
    elif args.legs != "none":
        legs = set(x.strip() for x in args.legs.split(",") if x.strip())
        if not legs <= {"config2", "config5"}:
            raise SystemExit("bench.py: --legs takes config2, config5, none or auto")

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: launch the ranks as children (this process has not touched the
        # GPU and never will: the devices are counted from the KFD topology, not through HIP) and exit with their
        # status.
        need = max(int(x) for x in args.device_of_rank.split(",")) + 1 if args.device_of_rank else args.gpus
        have = visible_gpu_count()
        if have is not None and have < need:
            raise SystemExit("bench.py: --gpus %d needs %d visible GPU(s), %d visible" % (args.gpus, need, have))
        return launch_ranks(args.gpus)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started %d rank(s)" % (args.gpus, world))

    if args.sites and args.taxa:
        import tempfile
        import gen_synthetic
        seed = 20261015 if (args.sites, args.taxa) == (256, 512) else 20261016
        args.dataset = os.path.join(tempfile.gettempdir(), "sr_synth_%dx%d_%d.txt" % (args.sites, args.taxa, seed))
        if not os.path.exists(args.dataset):
            gen_synthetic.write(args.sites, args.taxa, seed, args.dataset)
    elif not os.path.exists(args.dataset):
        import gen_synthetic
        gen_synthetic.write(256, 512, 20261015, args.dataset)

    total = args.chains_per_gpu * world if args.chains_per_gpu else args.total_chains
    if total < world:
        raise SystemExit("bench.py: %d chains cannot be sharded over %d GPUs" % (total, world))
    scaling = "weak" if args.chains_per_gpu else "strong"

    # CPU baseline and the CPU side of the extra legs first, before this process touches the GPU (they fork).
    cpu = cpu_o0 = c2cpu = None
    tmp = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        workers = args.cpu_workers or min(cpu_share()[0], total)
        warm_calls = args.warmup * args.calls_per_step
        cpu = cpu_baseline(args.dataset, warm_calls, args.cpu_calls, workers)
        cpu_o0 = cpu_baseline(args.dataset, warm_calls, max(1, args.cpu_calls // 4), workers, "O0")
        cpu_o0["kind"] = "port (reference-like -O0 build)"
    if rank == 0 and world == 1 and "config2" in legs:
        import tempfile
        tmp = tempfile.mkdtemp(prefix="sr_bench_c2_")
        if not args.no_cpu_baseline:
            c2cpu = leg_config2_cpu(args.cpu_workers or min(cpu_share()[0], 16), tmp)

    import numpy as np
    import torch
    import seriation_amd as sa
    from seriation_amd import dist as sd

    dist = None
    device = local_rank
    if args.device_of_rank:
        device = [int(x) for x in args.device_of_rank.split(",")][local_rank]
    torch.cuda.set_device(device)
    coll_dev = "cuda" if args.dist_backend == "nccl" else "cpu"   # where the end-of-run collectives' tensors live
    if "WORLD_SIZE" in os.environ:   # under a launcher: the RCCL path, also at world 1
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus, "torch.distributed world does not match --gpus"
        world = dist.get_world_size()

    # the session runs the sweep kernel compiled for this dataset's shape (the library's default for LDS
    # columns; cached, identical results) unless --generic
    ds = sa.Dataset.load(args.dataset, maxs=0)
    # rank r owns the contiguous block sd.shard(total, world, r) (ragged when world does not divide total), seed = id + 1
    chain_ids = list(sd.shard(total, world, rank))
    C = len(chain_ids)
    shards = [len(sd.shard(total, world, r)) for r in range(world)]
    seeds = [i + 1 for i in chain_ids]
    cps = args.calls_per_step
    # records of every timed step are kept (steps x calls-per-step saved samples per chain: 1000 at the
    # driver's --steps 20, the reference's sampling window ts = 1000, mcmc.c:180-185)
    sess = sa.Session(ds, seeds, device=device, calls_per_launch=max(1, args.steps * cps),
                      block_threads=args.block_threads, chain_ids=chain_ids, columns=args.columns, rng=args.rng,
                      generic=args.generic)
    stream = torch.cuda.current_stream()
    sess.set_stream(stream.cuda_stream)

    def step():
        sess.run(cps, save=not args.no_save)

    for _ in range(args.warmup):
        sess.run(cps, save=False)
    sess.reset_records()
    # device workspace of the selected chains' records (allocated before the timed region)
    nrec_ws = args.steps * cps if not args.no_save else 1
    rec_ws = sd.selected_records_workspace(CHAINS_SELECTED, nrec_ws, 2 * ds.M + ds.N, torch.device("cuda", device))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        evs[k][0].record(stream)
        step()
        evs[k][1].record(stream)
    if args.no_save:   # summaries from the final state (c, d, loglik) when no records were kept
        sess.reset_records()
        sess.run(1, save=True)
    stream.synchronize()
    t_kernels = time.perf_counter()
    # the end of the run: each chain's exp_data summary over its saved samples
    # (compute_exp_data, mcmc.c:53-67, in C) -> ONE all-gather of the summaries -> the one-sigma
    # selection on every rank -> the selected chains' saved samples gathered from their owners
    rows = sess.summaries()
    t_summ = time.perf_counter()
    nrec = int(sess.fetch_cdl().shape[1]) if args.no_save else args.steps * cps
    if dist:
        gathered = sd.gather_summaries(rows, total, device=coll_dev)
    else:
        gathered = rows
    selected = sd.select_chains(gathered, CHAINS_SELECTED)
    t_sel = time.perf_counter()
    W = 2 * ds.M + ds.N
    # the selected chains' records: device-to-device copies out of the session's record buffer on this stream,
    # then (N > 1) one all-gather per array over RCCL -- they never leave HBM inside the timed region
    dev_ab, dev_cd = sd.gather_selected_records_device(
        selected, total, chain_ids, lambda j, pa, pc: sess.copy_chain_records(j, pa, pc, count=nrec), nrec, W,
        device=torch.device("cuda", device), ws=rec_ws if nrec == nrec_ws else None)
    t_fetch = t_sel
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tail_ms = (time.perf_counter() - t_kernels) * 1e3
    tail_parts = {"summaries_ms": (t_summ - t_kernels) * 1e3, "gather_select_ms": (t_sel - t_summ) * 1e3,
                  "copy_gather_records_ms": (time.perf_counter() - t_fetch) * 1e3}
    sel_ab, sel_cdl = dev_ab.cpu().numpy(), dev_cd.cpu().numpy()   # (host copies for the statistics: untimed)
    # posterior statistics of the selected chains (script.py:100-152), outside the timed region
    ec, ed, corr = sd.selection_statistics(sel_ab, sel_cdl, ds.N, ds.M, CHAINS_SELECTED)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kernel_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    assert len(gathered) == total and np.isfinite(gathered).all() and selected
    assert sel_ab.shape[0] == len(selected) and (sel_ab[:, :, 2 * ds.M:] >= 0).all()

    sweeps_per_step = cps * 10
    iters = total * sweeps_per_step * args.steps
    value = iters / elapsed
    B = algorithmic_bytes_per_iter(ds.N, ds.M)
    launch_bytes = C * sweeps_per_step * B
    achieved = launch_bytes / (kernel_ms / 1e3) / 1e9
    traffic, traffic_src, prof = measured_traffic(ds.N, ds.M, C, sweeps_per_step)
    # what bounds the kernel, from the same PMC summary (SQ counters): the LDS-resident variant is
    # bound by per-wave issue and latency (its HBM traffic is the state and the records); the
    # HBM-column variant (columns too large for LDS, config 5) re-reads its columns from L2 / HBM
    limiter = dict(prof.get("limiter") or {})
    limiter["bound"] = ("issue / latency (working set in LDS; HBM carries only chain state and records)"
                        if sess.variant == "lds" else "L2 / MALL latency of the occurrence-column reads (columns in HBM, "
                        "re-read every sweep; HBM bandwidth far from peak)")
    limiter["source"] = traffic_src
    out = {
        # BASELINE.json's metric names the headline workload; any other shape or chain count says what it ran
        "metric": ("chain-iterations/sec (100 chains, 256x512 matrix) at 1/2/4/8 MI355X"
                   if (ds.N, ds.M, total) == (256, 512, 100) else
                   "chain-iterations/sec (%d chains, %dx%d matrix) at %d MI355X" % (total, ds.N, ds.M, world)),
        "value": value,
        "unit": "chain-iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": ("%s %dx%d, %d chains (%s), "
                         "%d mcmc_sample calls (%d sweeps) per chain per step, " +
                         ("no records saved" if args.no_save else "one saved record per call"))
                        % ("synthetic (tools/gen_synthetic.py seed %d)" % (20261015 if (ds.N, ds.M) == (256, 512)
                                                                          else 20261016)
                           if args.dataset == SYNTH or args.sites else os.path.basename(args.dataset),
                           ds.N, ds.M, total, ("%d per GPU" % C) if scaling == "weak" else
                           "sharded over %d GPU(s): %s" % (world, "/".join(map(str, shards))), cps, sweeps_per_step),
            "sites": ds.N, "taxa": ds.M, "chains": total, "chains_per_gpu": C, "chains_per_rank": shards,
            "scaling_mode": "strong: %d chains in total at every N" % total if scaling == "strong" else
                            "weak: %d chains per GPU" % C,
            "sweeps_per_step": sweeps_per_step, "block_threads": sess.block_threads, "columns": sess.variant,
            "kernel": sess.kernel,   # "split": two workgroups per chain (HBM columns)
            # split chains need both halves resident: hipLaunchCooperativeKernel (the product path), or an ordinary
            # launch of the same grid under SR_COOP=0 (the profiling runs: rocprofv3's tracer aborts at exit after
            # cooperative launches)
            "launch": ("ordinary (SR_COOP=0)" if os.environ.get("SR_COOP") == "0" else "cooperative")
                      if sess.kernel == "split" else "ordinary",
            "kernel_build": "specialized" if sess.specialized else "generic",   # the default is specialized
            "rng": "GSL MT19937 (the reference's stream)" if args.rng == "mt" else "Philox4x32-10 (opt-in)",
            "parallelism": "chains sharded over %d GPU(s), %s all-gather at end" % (
                world, "RCCL" if args.dist_backend == "nccl" else "gloo (host)"),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_unit": "bytes per launch (HBM, PMC)",
            "traffic_source": traffic_src,
            "kernel": "sr_sweep_kernel",
            "kernel_ms": kernel_ms,
            "bytes_per_chain_iteration": B,
            "launch_bytes": launch_bytes,
        },
        "limiter": limiter,
        "cpu_baseline": cpu,
        "cpu_baseline_O0": cpu_o0,
        "timing": {"kernel_ms_per_step": kernel_ms, "gather_select_ms": tail_ms, "tail_parts": tail_parts,
                   "note": "gather_select_ms: after the last kernel, the per-chain summaries (exp_data kernel), "
                           "their all-gather, the one-sigma selection, and the selected chains' records copied "
                           "device to device and all-gathered on the device (inside the timed region)"},
        "selection": {"chains_selected": selected, "exp_c": ec, "exp_d": ed, "corr_mn": corr,
                      "samples_per_chain": nrec,
                      "records_sha256": hashlib.sha256(np.ascontiguousarray(sel_ab).tobytes() +
                                                       np.ascontiguousarray(sel_cdl).tobytes()).hexdigest(),
                      "note": "script.py:70-152 over every timed step's saved samples of the selected chains (the "
                              "reference divides by 1000: exact means at --steps 20 x 50 calls = 1000 samples)"},
    }
    # parity leg inputs (outside the timed region, rank 0): besides the selected chains, chains the selection
    # rejected -- the first and the last of this rank's shard that were not selected -- so the check does not
    # sample only the best-loglik chains the records under test chose
    want_parity = rank == 0 and args.parity_chains > 0 and not args.no_save and args.rng == "mt"
    rej, rej_ab, rej_cd = [], None, None
    if want_parity and args.parity_rejected > 0:
        pool = [c for c in chain_ids if c not in set(selected)]
        pick = pool[:1] + pool[1:][-1:] if args.parity_rejected >= 2 else pool[:1]
        pick += [c for c in pool if c not in pick][:max(0, args.parity_rejected - len(pick))]
        rej = sorted(pick)
        rr = [sess.fetch_chain_records(chain_ids.index(c), count=nrec) for c in rej]
        if rr:
            rej_ab, rej_cd = np.stack([a for a, _ in rr]), np.stack([c for _, c in rr])
    variant = sess.variant
    sess.close()
    if dist:   # (the ranks leave together; rank 0's CPU parity leg below runs after the process group is gone)
        dist.destroy_process_group()
    # parity leg (after the timed region, rank 0): the CPU oracle reruns the checked chains and every compared
    # saved record of the timed region must match bit for bit (tests/bench_parity.py; the checker, not measured)
    parity = None
    if want_parity:
        import bench_parity
        with open(args.dataset, "rb") as fh:
            text = fh.read()
        k = min(args.parity_chains, len(selected))
        chk = list(selected[:k]) + rej
        ab = np.concatenate([sel_ab[:k]] + ([rej_ab] if rej else []))
        cd = np.concatenate([sel_cdl[:k]] + ([rej_cd] if rej else []))
        pc = args.parity_calls if args.parity_calls >= 0 else (0 if variant == "lds" else 4)
        parity = bench_parity.check_selected(text, chk, [c + 1 for c in chk], args.warmup * cps, ab, cd,
                                             calls=pc or None)
        parity["selected_checked"] = [int(c) for c in selected[:k]]
        parity["rejected_checked"] = [int(c) for c in rej]
        if pc:
            parity["calls_bound"] = ("--parity-calls %d" % pc if args.parity_calls > 0 else
                                     "auto: HBM-column session, the oracle takes ~0.4 s per call at this size")
    out["parity"] = parity
    # the extra workloads of the same line (N = 1, rank 0, after the headline and its parity leg)
    if rank == 0 and world == 1:
        if "config2" in legs:
            out["config2"] = leg_config2_gpu(device, tmp, c2cpu)
        if "config5" in legs:
            out["config5"] = leg_config5(device)
    if tmp:
        import shutil
        shutil.rmtree(tmp, ignore_errors=True)
    if rank == 0:
        print(json.dumps(out), flush=True)
    for leg in ("config2", "config5"):
        p = (out.get(leg) or {}).get("parity")
        if p is not None and not p["match"]:
            raise SystemExit("bench.py: %s differs from its oracle reference: %s" % (leg, p["mismatch"]))
    if parity is not None and not parity["match"]:
        raise SystemExit("bench.py: the timed records differ from the CPU oracle: %s" % parity["mismatch"])


if __name__ == "__main__":
    sys.exit(main())
