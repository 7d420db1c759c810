"""seriation_amd -- MI355X-native drop-in for the reference's per-chain MCMC sweep.

Layers (reference file in parentheses):
  _lib      ctypes binding of libseriation.so (C ABI: include/seriation.h)
  core      Dataset / Session / run_chains / run_to_dirs   (mcmc.c main + mcmc.h API)
  launcher  run_chain / run_all_chains / choose_chains     (script.py:15-99)
  dist      chain sharding + the one all-gather (RCCL)     (replaces script.py's Pool(8))
  analysis  E[c], E[d], CORRMN, pair-order matrix          (script.py:102-189)
"""
from ._lib import SrError, LIB_PATH, lib  # noqa: F401
from .core import Dataset, Session, run_chains, run_to_dirs, specialize  # noqa: F401
from . import launcher, analysis, dist  # noqa: F401

__all__ = ["Dataset", "Session", "run_chains", "run_to_dirs", "specialize", "launcher", "analysis", "dist", "SrError", "lib", "LIB_PATH"]
