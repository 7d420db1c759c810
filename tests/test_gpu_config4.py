"""BASELINE.json config 4 on one GPU: 800 chains of the synthetic 256x512 workload through the
shard path of the multi-GPU run (seriation_amd.dist.shard: 8 ranks x 100 chains, chain id =
global index, seed = id + 1), each shard its own session as each rank's would be.

* sharded == unsharded: every chain's saved samples are identical whether it runs in its
  shard's 100-chain session or in one 800-chain session;
* 8 chains spread over the shards are bit-exact against the CPU oracle for 20 calls.
(script.py:55-62 runs chains independently)"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle_ref
import seriation_amd as sa
from seriation_amd import dist as sd

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
SYNTH = os.path.join(HERE, "golden", "datasets", "synth_256x512.txt")
WORLD, PER = 8, 100
CALLS = 20


@pytest.fixture(scope="module")
def config4():
    ds = sa.Dataset.load(SYNTH, maxs=0)
    total = WORLD * PER
    shard_ab, shard_cdl, shard_ids = [], [], []
    for r in range(WORLD):
        ids = list(sd.shard(total, WORLD, r))
        with sa.Session(ds, [i + 1 for i in ids], chain_ids=ids, calls_per_launch=CALLS) as s:
            s.run(CALLS, save=True)
            ab, cdl = s.fetch_records()
        shard_ab.append(ab)
        shard_cdl.append(cdl)
        shard_ids += ids
    ids = list(range(total))
    with sa.Session(ds, [i + 1 for i in ids], chain_ids=ids, calls_per_launch=CALLS) as s:
        s.run(CALLS, save=True)
        ab_all, cdl_all = s.fetch_records()
    return ds, shard_ids, np.concatenate(shard_ab), np.concatenate(shard_cdl), ab_all, cdl_all


def test_shards_cover_config4(config4):
    ds, ids, ab, cdl, ab_all, cdl_all = config4
    assert ids == list(range(WORLD * PER))
    assert ab.shape == (WORLD * PER, CALLS, 2 * ds.M + ds.N)


def test_sharded_equals_unsharded(config4):
    ds, ids, ab, cdl, ab_all, cdl_all = config4
    assert np.array_equal(ab, ab_all)
    assert np.array_equal(cdl.view(np.uint64), cdl_all.view(np.uint64))


def test_spread_chains_match_oracle(config4):
    ds, ids, ab, cdl, ab_all, cdl_all = config4
    with open(SYNTH, "rb") as fh:
        text = fh.read()
    picks = [0, 105, 211, 317, 422, 528, 634, 799]   # one chain in every shard

    def one(i):
        o = oracle_ref.run_chain(text, i + 1, 0, CALLS, maxs=0)
        return o["rc"], o["rec_int"].copy(), o["rec_dbl"].copy()

    with ThreadPoolExecutor(8) as ex:
        ref = list(ex.map(one, picks))
    for i, (rc, ri, rdb) in zip(picks, ref):
        assert rc == 0
        assert np.array_equal(ab[i].astype(np.int32), ri), "chain %d: integers differ from the oracle" % i
        assert np.array_equal(cdl[i].view(np.uint64), rdb.view(np.uint64)), "chain %d: c/d/loglik differ" % i
