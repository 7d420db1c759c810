"""Pythonic wrappers over the C ABI: datasets, sessions, whole-run helpers.

These mirror the reference's C entry points (C_Implementation/mcmc.h:47-72) with numpy
arrays instead of gsl containers; the computation always happens in libseriation.so on
the GPU.
"""
import ctypes
import os

import numpy as np

from . import _lib as L


def _check(rc, what):
    if rc != L.SR_OK:
        raise L.SrError(rc, what)


class Dataset:
    """Occurrence matrix X (N sites x M taxa, uint8 0/1) and hard-site flags.

    Parsed exactly like mcmc_readmodel (mcmc.c:339-437); ``maxs=2000`` keeps the
    reference's fgets(MAXS) line limit, ``maxs=0`` accepts lines of any length.
    """

    def __init__(self, X, hard):
        self.X = np.ascontiguousarray(X, dtype=np.uint8)
        self.hard = np.ascontiguousarray(hard, dtype=np.uint8)
        assert self.X.ndim == 2 and self.hard.shape == (self.X.shape[0],)
        self.N, self.M = self.X.shape
        self.nh = int(self.hard.sum())
        self._c = L.sr_dataset(self.N, self.M, self.nh,
                               self.X.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                               self.hard.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))

    @classmethod
    def parse(cls, text, maxs=L.SR_MAXS):
        if isinstance(text, str):
            text = text.encode()
        ds = L.sr_dataset()
        _check(L.lib().sr_parse_dataset(text, len(text), maxs, ctypes.byref(ds)), "parse")
        return cls._adopt(ds)

    @classmethod
    def _adopt(cls, ds):
        try:
            X = np.ctypeslib.as_array(ds.X, shape=(ds.N * ds.M,)).reshape(ds.N, ds.M).copy()
            hard = np.ctypeslib.as_array(ds.hard, shape=(ds.N,)).copy()
        finally:
            L.lib().sr_free_dataset(ctypes.byref(ds))
        return cls(X, hard)

    @classmethod
    def load(cls, path, maxs=L.SR_MAXS):
        ds = L.sr_dataset()
        _check(L.lib().sr_load_dataset(os.fsencode(path), maxs, ctypes.byref(ds)), "load %s" % path)
        return cls._adopt(ds)

    def save_bin(self, path):
        """Write the bit-packed binary form (sr_save_dataset_bin)."""
        _check(L.lib().sr_save_dataset_bin(ctypes.byref(self._c), os.fsencode(path)), "save_bin %s" % path)

    @classmethod
    def load_bin(cls, path):
        ds = L.sr_dataset()
        _check(L.lib().sr_load_dataset_bin(os.fsencode(path), ctypes.byref(ds)), "load_bin %s" % path)
        return cls._adopt(ds)

    @property
    def c(self):
        return self._c


def make_opts(burnin_calls=1000, sample_calls=1000, sweeps_per_call=10, device=0, block_threads=0,
              calls_per_launch=0, check=True, columns="auto", debug_check=False, debug_print=False, rng="mt",
              generic=False, manycd=0):
    """columns: "auto" (LDS when the layout fits, else HBM), "lds" or "hbm" (SR_F_*_COLUMNS).
    debug_check: mcmc_consistent after every mcmc_sample call (the reference's MCMCDEBUG,
    mcmc.c:249-255; SR_F_DEBUG_CHECK), debug_print: its acceptance-rate lines on stderr.
    rng: "mt" (the reference's GSL MT19937 stream, bit-exact) or "philox" (opt-in SR_F_RNG_PHILOX:
    counter-based Philox4x32-10 per chain for the sampling phase; statistically equivalent only).
    generic: the generic sweep kernel instead of the default shape-specialised one (SR_F_GENERIC_KERNEL;
    identical results).  manycd: 1 = per-taxon c[m], d[m] (mcmc_readmodel's manycd, mcmc.c:777-786, 807-816)."""
    o = L.sr_run_opts()
    L.lib().sr_default_opts(ctypes.byref(o))
    o.burnin_calls = burnin_calls
    o.sample_calls = sample_calls
    o.sweeps_per_call = sweeps_per_call
    o.device = device
    o.block_threads = block_threads
    o.calls_per_launch = calls_per_launch
    o.manycd = 1 if manycd else 0
    o.flags = (0 if check else L.SR_F_NO_CHECK) | {"auto": 0, "lds": L.SR_F_LDS_COLUMNS,
                                                   "hbm": L.SR_F_HBM_COLUMNS}[columns]
    if debug_check:
        o.flags |= L.SR_F_DEBUG_CHECK | (L.SR_F_DEBUG_PRINT if debug_print else 0)
    if rng not in ("mt", "philox"):
        raise ValueError("rng must be 'mt' or 'philox'")
    if rng == "philox":
        o.flags |= L.SR_F_RNG_PHILOX
    if generic:
        o.flags |= L.SR_F_GENERIC_KERNEL
    return o


def specialize(dataset, block_threads=0, columns="auto"):
    """sr_specialize: compile (or find cached) the shape-specialised sweep kernel a session over `dataset`
    would run, without a GPU.  True: ready; False: such a session runs no specialised kernel (HBM columns)."""
    o = make_opts(block_threads=block_threads, columns=columns)
    rc = L.lib().sr_specialize(ctypes.byref(dataset.c), ctypes.byref(o))
    if rc < 0:
        raise L.SrError(rc, "sr_specialize")
    return rc == 1


def make_specs(seeds, chain_ids=None):
    n = len(seeds)
    arr = (L.sr_chain_spec * n)()
    for k, s in enumerate(seeds):
        arr[k].chain_id = int(chain_ids[k]) if chain_ids is not None else k
        arr[k].seed = int(s)
    return arr


class Session:
    """Chains resident on one GPU (sr_session_*).  ``run(calls, save)`` enqueues
    ``calls`` mcmc_sample calls (mcmc.c:214-258) for every chain."""

    def __init__(self, dataset, seeds, device=0, sweeps_per_call=10, calls_per_launch=0, block_threads=0,
                 chain_ids=None, columns="auto", debug_check=False, rng="mt", generic=False, manycd=0):
        self.ds = dataset
        self.n = len(seeds)
        self.specs = make_specs(seeds, chain_ids)
        self.opts = make_opts(sweeps_per_call=sweeps_per_call, device=device, block_threads=block_threads,
                              calls_per_launch=calls_per_launch, columns=columns, debug_check=debug_check, rng=rng,
                              generic=generic, manycd=manycd)
        h = ctypes.c_void_p()
        _check(L.lib().sr_session_create(ctypes.byref(dataset.c), self.specs, self.n, ctypes.byref(self.opts),
                                         ctypes.byref(h)), "sr_session_create")
        self.h = h

    def checkpoint(self, path):
        """sr_session_checkpoint: the full chain state and the buffered records to `path`."""
        _check(L.lib().sr_session_checkpoint(self.h, os.fsencode(path)), "sr_session_checkpoint")

    @classmethod
    def restore(cls, dataset, path, device=0, sweeps_per_call=10, calls_per_launch=0, block_threads=0,
                columns="auto", rng="mt", manycd=0):
        """sr_session_restore: a session continuing the chains of a checkpoint over `dataset` (manycd must
        name the checkpoint's kind)."""
        self = cls.__new__(cls)
        self.ds = dataset
        self.opts = make_opts(sweeps_per_call=sweeps_per_call, device=device, block_threads=block_threads,
                              calls_per_launch=calls_per_launch, columns=columns, rng=rng, manycd=manycd)
        h = ctypes.c_void_p()
        _check(L.lib().sr_session_restore(ctypes.byref(dataset.c), os.fsencode(path), ctypes.byref(self.opts),
                                          ctypes.byref(h)), "sr_session_restore")
        self.h = h
        with open(path, "rb") as fh:   # header: magic, version, N, M, nh, nchains
            self.n = int(np.frombuffer(fh.read(24)[20:24], "<i4")[0])
        self.specs = None
        return self

    @property
    def record_capacity(self):
        return L.lib().sr_session_record_capacity(self.h)

    @property
    def block_threads(self):
        return L.lib().sr_session_block_threads(self.h)

    @property
    def variant(self):
        """Kernel variant: "lds" (occurrence columns in LDS) or "hbm" (columns in HBM)."""
        return "hbm" if L.lib().sr_session_variant(self.h) in (1, 3) else "lds"

    @property
    def kernel(self):
        """"pair" (two lanes per taxon), "split" (HBM columns, two workgroups per chain) or "single"
        (one workgroup per chain, one thread per taxon or several)."""
        return {2: "pair", 3: "split"}.get(L.lib().sr_session_variant(self.h), "single")

    @property
    def specialized(self):
        """True when the launches use the sweep kernel compiled for this dataset's exact shape (the default
        for LDS-column sessions), False for the generic one (HBM columns, generic=True,
        SR_JIT=0 in the environment, or the specialised code object unavailable)."""
        return bool(L.lib().sr_session_specialized(self.h))

    def set_stream(self, stream_handle):
        _check(L.lib().sr_session_set_stream(self.h, ctypes.c_void_p(stream_handle)), "set_stream")

    def run(self, calls, save=False):
        _check(L.lib().sr_session_run(self.h, calls, 1 if save else 0), "sr_session_run")

    def sync(self):
        _check(L.lib().sr_session_sync(self.h), "sr_session_sync")

    def last_kernel_ms(self):
        return L.lib().sr_session_last_kernel_ms(self.h)

    def reset_records(self):
        _check(L.lib().sr_session_reset_records(self.h), "reset_records")

    def fetch_records(self):
        """Returns (ab_pi int16 [n, k, 2M+N], cdl float64 [n, k, 3]) for the k buffered calls."""
        k = L.lib().sr_session_records(self.h)
        N, M = self.ds.N, self.ds.M
        ab = np.zeros((self.n, k, 2 * M + N), np.int16)
        cdl = np.zeros((self.n, k, 3), np.float64)
        if k:
            _check(L.lib().sr_session_fetch_records(self.h, 0, k, ab.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)),
                                                    cdl.ctypes.data_as(ctypes.POINTER(ctypes.c_double))), "fetch")
        return ab, cdl

    @property
    def manycd(self):
        return bool(L.lib().sr_session_manycd(self.h))

    def fetch_cd_vectors(self):
        """manycd sessions: every taxon's (c, d) of the k buffered calls, float64 [n, k, 2M] (c[M] then d[M])."""
        k = L.lib().sr_session_records(self.h)
        cv = np.zeros((self.n, k, 2 * self.ds.M), np.float64)
        if k:
            _check(L.lib().sr_session_fetch_cd_vectors(self.h, 0, k, cv.ctypes.data_as(ctypes.POINTER(ctypes.c_double))),
                   "fetch_cd_vectors")
        return cv

    def fetch_cdl(self):
        """(c, d, loglik) float64 [n, k, 3] of the k buffered calls, without the a/b/pi rows."""
        k = L.lib().sr_session_records(self.h)
        cdl = np.zeros((self.n, k, 3), np.float64)
        if k:
            _check(L.lib().sr_session_fetch_records(self.h, 0, k, None,
                                                    cdl.ctypes.data_as(ctypes.POINTER(ctypes.c_double))), "fetch")
        return cdl

    def fetch_chain_records(self, chain, first=0, count=None, out=None):
        """One chain's buffered records: (ab_pi int16 [count, 2M+N], cdl float64 [count, 3]); out: a
        caller-owned pair of C-contiguous arrays of those shapes to fill (e.g. views of pinned host
        memory, so the copy runs at DMA speed without page faults)."""
        k = L.lib().sr_session_records(self.h)
        count = k - first if count is None else count
        N, M = self.ds.N, self.ds.M
        if out is not None:
            ab, cdl = out
            if ab.shape != (count, 2 * M + N) or ab.dtype != np.int16 or not ab.flags.c_contiguous or \
                    cdl.shape != (count, 3) or cdl.dtype != np.float64 or not cdl.flags.c_contiguous:
                raise ValueError("fetch_chain_records: out arrays must be C-contiguous int16 [%d, %d] and "
                                 "float64 [%d, 3]" % (count, 2 * M + N, count))
        else:
            ab = np.zeros((count, 2 * M + N), np.int16)
            cdl = np.zeros((count, 3), np.float64)
        if count:
            _check(L.lib().sr_session_fetch_chain_records(self.h, chain, first, count,
                                                          ab.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)),
                                                          cdl.ctypes.data_as(ctypes.POINTER(ctypes.c_double))),
                   "fetch_chain_records")
        return ab, cdl

    def copy_chain_records(self, chain, ab_ptr, cdl_ptr, first=0, count=None):
        """sr_session_copy_chain_records: one chain's buffered records copied device to device, queued on the
        session stream, into device memory at ab_ptr ([count, 2M+N] int16) / cdl_ptr ([count, 3] float64)
        (raw device addresses, e.g. a torch tensor's data_ptr(); 0 skips that array)."""
        k = L.lib().sr_session_records(self.h)
        count = k - first if count is None else count
        _check(L.lib().sr_session_copy_chain_records(self.h, chain, first, count, ctypes.c_void_p(ab_ptr or None),
                                                      ctypes.c_void_p(cdl_ptr or None)), "copy_chain_records")
        return count

    def summaries(self, first=0, count=None):
        """sr_session_summaries: exp_data rows (chain_id, exp_loglik, exp_c, exp_d) [n, 4] of every chain
        over its buffered records (mcmc.c:53-67; divisor 1000 as the reference)."""
        k = L.lib().sr_session_records(self.h)
        count = k - first if count is None else count
        out = (L.sr_chain_summary * self.n)()
        _check(L.lib().sr_session_summaries(self.h, first, count, out), "sr_session_summaries")
        return np.array([(o.chain_id, o.exp_loglik, o.exp_c, o.exp_d) for o in out], np.float64).reshape(self.n, 4)

    def state(self, chain):
        N, M = self.ds.N, self.ds.M
        a = np.zeros(M, np.int32)
        b = np.zeros(M, np.int32)
        pi = np.zeros(N, np.int32)
        cdl = np.zeros(3, np.float64)
        cnt = np.zeros(4 * M, np.int32)
        P = ctypes.POINTER
        _check(L.lib().sr_session_state(self.h, chain, a.ctypes.data_as(P(ctypes.c_int32)),
                                        b.ctypes.data_as(P(ctypes.c_int32)), pi.ctypes.data_as(P(ctypes.c_int32)),
                                        cdl.ctypes.data_as(P(ctypes.c_double)), cnt.ctypes.data_as(P(ctypes.c_int32))),
               "state")
        out = {"a": a, "b": b, "pi": pi, "c": cdl[0], "d": cdl[1], "loglik": cdl[2], "counts": cnt.reshape(4, M)}
        if self.manycd:   # every taxon's own c, d
            cv, dv = np.zeros(M), np.zeros(M)
            _check(L.lib().sr_session_state_cd(self.h, chain, cv.ctypes.data_as(P(ctypes.c_double)),
                                               dv.ctypes.data_as(P(ctypes.c_double))), "state_cd")
            out["cv"], out["dv"] = cv, dv
        return out

    def accept_counts(self, chain):
        acc = np.zeros(7, np.int64)
        _check(L.lib().sr_session_accept_counts(self.h, chain, acc.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))),
               "accept_counts")
        return acc

    def fallback_counts(self, chain):
        """sr_session_fallback_counts: {exact sequential deltas, exact Gibbs walks, sequential c/d
        draws} taken by `chain` so far."""
        fb = np.zeros(3, np.int64)
        _check(L.lib().sr_session_fallback_counts(self.h, chain, fb.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))),
               "fallback_counts")
        return fb

    def close(self):
        if self.h:
            L.lib().sr_session_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def _devices(devices):
    arr = (ctypes.c_int32 * len(devices))(*[int(d) for d in devices])
    return arr, len(devices)


def run_chains(dataset, seeds, burnin_calls=1000, sample_calls=1000, sweeps_per_call=10, device=0,
               chain_ids=None, keep_records=False, calls_per_launch=0, block_threads=0, columns="auto",
               devices=None, debug_check=False, rng="mt", generic=False, manycd=0):
    """sr_run_chains: returns (summaries list of dicts, records or None).
    records = (ab_pi int32 [n, ts, 2M+N], cdl [n, ts, 3]) when keep_records, plus cdv [n, ts, 2M] (every
    taxon's c then d) for manycd=1.
    devices: a list of HIP ordinals (may repeat) -> sr_run_chains_multi, chains sharded over them."""
    n = len(seeds)
    specs = make_specs(seeds, chain_ids)
    opts = make_opts(burnin_calls, sample_calls, sweeps_per_call, device, block_threads=block_threads,
                     calls_per_launch=calls_per_launch, columns=columns, debug_check=debug_check, rng=rng,
                     generic=generic, manycd=manycd)
    out = (L.sr_chain_summary * n)()
    N, M = dataset.N, dataset.M
    recs = None
    if keep_records:
        recs = (np.zeros((n, sample_calls, 2 * M + N), np.int32), np.zeros((n, sample_calls, 3)))
        if manycd:
            recs = recs + (np.zeros((n, sample_calls, 2 * M)),)

    def sink(ctx, ci, si, rp):
        r = rp.contents
        ab = recs[0][ci, si]
        ab[:M] = np.ctypeslib.as_array(r.a, shape=(M,))
        ab[M:2 * M] = np.ctypeslib.as_array(r.b, shape=(M,))
        ab[2 * M:] = np.ctypeslib.as_array(r.pi, shape=(N,))
        recs[1][ci, si] = (r.c, r.d, r.loglik)
        if manycd:
            recs[2][ci, si, :M] = np.ctypeslib.as_array(r.cv, shape=(M,))
            recs[2][ci, si, M:] = np.ctypeslib.as_array(r.dv, shape=(M,))
        return 0

    cb = L.SINK_FN(sink) if keep_records else ctypes.cast(None, L.SINK_FN)
    if devices:
        darr, nd = _devices(devices)
        rc = L.lib().sr_run_chains_multi(ctypes.byref(dataset.c), specs, n, ctypes.byref(opts), darr, nd, cb, None, out)
    else:
        rc = L.lib().sr_run_chains(ctypes.byref(dataset.c), specs, n, ctypes.byref(opts), cb, None, out)
    if rc not in (L.SR_OK, L.SR_EINCONSISTENT):
        raise L.SrError(rc, "sr_run_chains")
    summ = [dict(chain_id=o.chain_id, consistent=o.consistent, exp_loglik=o.exp_loglik, exp_c=o.exp_c,
                 exp_d=o.exp_d) for o in out]
    return summ, recs


def run_to_dirs(dataset, seeds, root=".", chain_ids=None, burnin_calls=1000, sample_calls=1000, device=0,
                sweeps_per_call=10, devices=None, rng="mt", manycd=0):
    """sr_run_to_dirs: writes Chains/chain_NN/*.csv under root like the reference main().
    sweeps_per_call is the thinning (the reference's mcmc_sample runs 10, mcmc.c:225).
    devices: HIP ordinals (may repeat) -> sr_run_to_dirs_multi."""
    n = len(seeds)
    specs = make_specs(seeds, chain_ids)
    opts = make_opts(burnin_calls, sample_calls, sweeps_per_call, device, rng=rng, manycd=manycd)
    out = (L.sr_chain_summary * n)()
    if devices:
        darr, nd = _devices(devices)
        rc = L.lib().sr_run_to_dirs_multi(ctypes.byref(dataset.c), specs, n, ctypes.byref(opts), darr, nd,
                                          os.fsencode(root), out)
    else:
        rc = L.lib().sr_run_to_dirs(ctypes.byref(dataset.c), specs, n, ctypes.byref(opts),
                                    os.fsencode(root), out)
    if rc not in (L.SR_OK, L.SR_EINCONSISTENT):
        raise L.SrError(rc, "sr_run_to_dirs")
    return [dict(chain_id=o.chain_id, consistent=o.consistent, exp_loglik=o.exp_loglik, exp_c=o.exp_c,
                 exp_d=o.exp_d) for o in out]
