"""bench.py's parity leg (tests/bench_parity.py) on the CPU: records equal to the oracle's pass, and a single
flipped bit -- an integer of one saved sample, or the last bit of one loglik -- is reported for that chain and
call.  (On the GPU the leg checks the bench's own timed records: tests/test_gpu_rccl.py, BENCH lines.)"""
import os

import numpy as np

import bench_parity
import oracle_ref

HERE = os.path.dirname(os.path.abspath(__file__))


def _records(text, seeds, tb, ts):
    ab, cd = [], []
    for s in seeds:
        o = oracle_ref.run_chain(text, s, tb, ts)
        ab.append(o["rec_int"].astype(np.int16))
        cd.append(o["rec_dbl"])
    return np.stack(ab), np.stack(cd)


def test_parity_leg_matches_and_reports_mismatches():
    with open(os.path.join(HERE, "golden", "datasets", "g10s10.txt"), "rb") as fh:
        text = fh.read()
    chains, seeds = [4, 9], [5, 10]
    ab, cd = _records(text, seeds, 3, 5)
    ok = bench_parity.check_selected(text, chains, seeds, 3, ab, cd, maxs=2000)
    assert ok["match"] and ok["saved_calls_compared"] == 5 and ok["mismatch"] == {}
    bad_ab = ab.copy()
    bad_ab[1, 2, 7] += 1
    r = bench_parity.check_selected(text, chains, seeds, 3, bad_ab, cd, maxs=2000)
    assert not r["match"] and list(r["mismatch"]) == ["9"] and "saved call 2" in r["mismatch"]["9"]
    bad_cd = cd.copy()
    bad_cd.view(np.uint64)[0, 4, 2] ^= 1
    r = bench_parity.check_selected(text, chains, seeds, 3, ab, bad_cd, maxs=2000)
    assert not r["match"] and list(r["mismatch"]) == ["4"] and "c/d/loglik" in r["mismatch"]["4"]
    # a prefix of the saved calls (the HBM-column workloads)
    r = bench_parity.check_selected(text, chains, seeds, 3, bad_ab, cd, calls=2, maxs=2000)
    assert r["match"] and r["saved_calls_compared"] == 2
