#!/usr/bin/env python3
"""Regenerate the committed golden fixtures under tests/golden/ (TEST INFRASTRUCTURE).

The reference ships no fixtures for the sampler (its Chains/ tree is empty placeholders,
SURVEY.md §4) and its binary cannot run here (GSL absent), so the vectors
below come from the CPU oracle (oracle/om_mcmc.c).  Independent pins are asserted by
tests/test_oracle_rng.py (mt19937 against numpy.random.RandomState, GSL sampling
semantics restated in Python); these files freeze the oracle's end-to-end output so the
GPU path can be checked against them on the box without re-running the oracle, and so a
change of the oracle shows up as a fixture diff.

    python tests/golden/make_golden.py        # rewrites mt19937.json and chains.json
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_ref  # noqa: E402

DS = os.path.join(HERE, "datasets")
MT_SEEDS = [0, 1, 42, 255, 4357]
MT_WORDS = 64
# (dataset, seeds, calls): per-call hashes of the first `calls` mcmc_sample calls
CHAIN_CASES = [("g2s2.txt", [1, 2, 3, 4], 30), ("g10s10.txt", [1, 2, 3, 4], 50),
               ("g5s5.txt", [1], 20), ("g10s2.txt", [1], 20), ("synth_256x512.txt", [1], 5)]


def record_digest(rec_int):
    """SHA-256 of a saved sample's pi || a || b (int32 little endian)."""
    return hashlib.sha256(np.ascontiguousarray(rec_int, dtype="<i4").tobytes()).hexdigest()


def chain_fixture(name, seed, calls):
    with open(os.path.join(DS, name), "rb") as fh:
        text = fh.read()
    o = oracle_ref.run_chain(text, seed, 0, calls, sweeps=10, check=1)
    assert o["rc"] == 0, (name, seed, o["rc"])
    return {
        "dataset": name, "seed": seed, "calls": calls, "N": int(o["N"]), "M": int(o["M"]),
        "init_sha256": record_digest(o["init"]),
        "init_cdl_hex": [float(v).hex() for v in o["init_cdl"]],
        "sha256": [record_digest(r) for r in o["rec_int"]],
        "cdl_hex": [[float(v).hex() for v in r] for r in o["rec_dbl"]],
        "exp_hex": [float(v).hex() for v in o["exp"]],
        "rng_words": int(o["words"]),
    }


def main():
    mt = {}
    for s in MT_SEEDS:
        w, _ = oracle_ref.rng_stream(s, 0, MT_WORDS)
        mt[str(s)] = [int(v) for v in w]
    with open(os.path.join(HERE, "mt19937.json"), "w") as fh:
        json.dump({"note": "gsl_rng_mt19937 raw words (seed 0 -> 4357), first %d per seed" % MT_WORDS,
                   "words": mt}, fh, indent=0)
    cases = [chain_fixture(n, s, c) for n, seeds, c in CHAIN_CASES for s in seeds]
    with open(os.path.join(HERE, "chains.json"), "w") as fh:
        json.dump({"note": "oracle per-call digests: sha256(a||b||pi int32le), c[0]/d[0]/loglik hex, "
                           "exp_data (/1000) hex; tb=0, 10 sweeps per call", "cases": cases}, fh, indent=1)
    print("wrote %d mt seeds, %d chain cases" % (len(mt), len(cases)))


if __name__ == "__main__":
    main()
