"""bench.py's parity leg -- TEST INFRASTRUCTURE (the checker, never the thing measured).

After bench.py's timed region, the CPU oracle (oracle/, the C restatement of mcmc.c) reruns some of the
chains the one-sigma selection kept -- same dataset, same seed, the bench's warm-up calls as burn-in, then
the saved calls -- and every saved record the GPU produced inside the timed region must equal the
oracle's bit for bit (a, b, pi as integers; c, d, loglik as f64 bits).  Reference: mcmc.c:140-185 (burn-in
then ts saved mcmc_sample calls).  The oracle chains run in threads (the ctypes call releases the GIL).
"""
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import oracle_ref


def check_selected(text, chains, seeds, burnin_calls, rec_ab, rec_cdl, calls=None, maxs=0):
    """chains/seeds: the checked chains' ids and GSL seeds; rec_ab [len(chains), S, 2M+N] int16 and rec_cdl
    [len(chains), S, 3] f64: their saved records from the timed region.  calls: compare the first `calls` of
    the S records (default all).  Returns the line's "parity" object."""
    S = rec_ab.shape[1]
    calls = S if calls is None else min(int(calls), S)
    oracle_ref.lib()
    t0 = time.perf_counter()

    def one(k):
        o = oracle_ref.run_chain(text, int(seeds[k]), int(burnin_calls), calls, sweeps=10, maxs=maxs)
        if o["rc"] != 0:
            return k, "oracle rc %d" % o["rc"]
        gi = rec_ab[k, :calls].astype(np.int32)
        bad = np.nonzero((gi != o["rec_int"]).any(axis=1))[0]
        if len(bad):
            return k, "integer state differs from saved call %d on" % int(bad[0])
        gd = np.ascontiguousarray(rec_cdl[k, :calls]).view(np.uint64)
        bad = np.nonzero((gd != o["rec_dbl"].view(np.uint64)).any(axis=1))[0]
        if len(bad):
            return k, "c/d/loglik bits differ from saved call %d on" % int(bad[0])
        return k, None

    with ThreadPoolExecutor(max_workers=max(1, len(chains))) as ex:
        res = dict(ex.map(one, range(len(chains))))
    return {"chains": [int(c) for c in chains], "seeds": [int(s) for s in seeds], "burnin_calls": int(burnin_calls),
            "saved_calls_compared": calls, "match": all(v is None for v in res.values()),
            "mismatch": {str(int(chains[k])): v for k, v in res.items() if v is not None},
            "oracle_wall_s": time.perf_counter() - t0,
            "note": "CPU oracle (oracle/om_mcmc.c) rerun of these selected chains after the timed region: every "
                    "compared saved record equal bit for bit (integers and f64 bits)"}
