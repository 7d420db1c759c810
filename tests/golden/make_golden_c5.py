#!/usr/bin/env python3
"""Config-5 golden fixtures: the converged regime of 1024 sites x 2048 taxa (TEST INFRASTRUCTURE).

BASELINE.json configs[4] (tools/gen_synthetic.py 1024 2048, seed 20261016, 12 hard sites) under the
reference CLI's own protocol, mcmc.c:140-185: 1000 burn-in calls of mcmc_sample (10 sweeps each, no
records), then 1000 saved calls -- 20 000 sweeps per chain, well past the ~10 000 sweeps where the
config-5 rates are quoted.  The CPU oracle (oracle/om_mcmc.c, parsed with maxs = 0 since the
reference's MAXS = 2000 cannot hold the 4096-char lines) writes per saved call:
  - sha256 of pi || a || b (int32 little endian, the record layout of chains.json),
  - c, d, loglik as float.hex,
and per chain exp_data (mcmc.c:53-67, over the 1000 saved calls) as hex.

These vectors reach the long-walk window trim (SR_QSPAN), the grouped f64 Gibbs checkpoints and the
LDS checkpoints of the split kernel at depth, which the GPU test tests/test_gpu_config5_golden.py
compares against without re-running the oracle on the box (~15 min of oracle time, 4 chains on 4
threads here).

    python tests/golden/make_golden_c5.py          # writes tests/golden/config5.json
"""
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_synthetic  # noqa: E402
import oracle_ref  # noqa: E402

SHAPE = (1024, 2048, 20261016)
SEEDS = [1, 2, 3, 4]
BURNIN, SAVED = 1000, 1000
OUT = os.path.join(HERE, "config5.json")


def dataset_text():
    X, hard = gen_synthetic.make(*SHAPE)
    return gen_synthetic.to_text(X, hard).encode()


def record_digest(rec_int):
    return hashlib.sha256(np.ascontiguousarray(rec_int, dtype="<i4").tobytes()).hexdigest()


def one(text, seed):
    t0 = time.time()
    o = oracle_ref.run_chain(text, seed, BURNIN, SAVED, sweeps=10, check=0, maxs=0)
    assert o["rc"] == 0, (seed, o["rc"])
    return {
        "seed": seed,
        "sha256": [record_digest(r) for r in o["rec_int"]],
        "cdl_hex": [[float(v).hex() for v in r] for r in o["rec_dbl"]],
        "exp_hex": [float(v).hex() for v in o["exp"]],
        "acc": [int(v) for v in o["acc"]],
        "rng_words": int(o["words"]),
        "oracle_s": round(time.time() - t0, 1),
    }


def main():
    text = dataset_text()
    with ThreadPoolExecutor(len(SEEDS)) as ex:
        chains = list(ex.map(lambda s: one(text, s), SEEDS))
    doc = {
        "note": "oracle/om_mcmc.c on tools/gen_synthetic.py %d %d seed %d (maxs=0): per saved call "
                "sha256(pi||a||b int32le), c/d/loglik hex; exp_data hex; %d burn-in + %d saved calls of "
                "10 sweeps (mcmc.c:140-185)" % (SHAPE + (BURNIN, SAVED)),
        "dataset_sha256": hashlib.sha256(text).hexdigest(),
        "N": SHAPE[0], "M": SHAPE[1], "gen_seed": SHAPE[2],
        "burnin_calls": BURNIN, "saved_calls": SAVED, "chains": chains,
    }
    with open(OUT, "w") as fh:
        json.dump(doc, fh, indent=0)
    print("wrote %s: %d chains, oracle %s s" % (OUT, len(chains), [c["oracle_s"] for c in chains]))


if __name__ == "__main__":
    main()
