#!/usr/bin/env python3
"""Synthetic seriation datasets, reference text format.

True order = row order.  Taxon m is born at a ~ U{0..N-1} and lives L ~ U{N/32..N/4}
sites, alive = [a, min(N, a+L)); X = 1 w.p. 0.5 inside (d_true = 0.5) and w.p. 0.01
outside (c_true = 0.01); all-zero columns are resampled; 12 hard sites ('*') at rows
floor((k+0.5) N/12).  Lines are "0 1 0 ... *" like Dataset/*.txt.

  python tools/gen_synthetic.py N M SEED OUT
"""
import hashlib
import os
import sys

import numpy as np


def make(N, M, seed, n_hard=12):
    rng = np.random.default_rng(seed)
    X = np.zeros((N, M), np.uint8)
    for m in range(M):
        while True:
            a = rng.integers(0, N)
            L = rng.integers(max(1, N // 32), max(2, N // 4) + 1)
            b = min(N, a + L)
            col = (rng.random(N) < 0.01).astype(np.uint8)
            col[a:b] = (rng.random(b - a) < 0.5).astype(np.uint8)
            if col.any():
                X[:, m] = col
                break
    hard = np.zeros(N, np.uint8)
    for k in range(n_hard):
        hard[int((k + 0.5) * N / n_hard)] = 1
    return X, hard


def to_text(X, hard):
    N, M = X.shape
    lines = ["%d %d" % (N, M)]
    for i in range(N):
        row = " ".join("1" if v else "0" for v in X[i])
        lines.append(row + (" *" if hard[i] else ""))
    return "\n".join(lines) + "\n"


def write(N, M, seed, out):
    X, hard = make(N, M, seed)
    txt = to_text(X, hard)
    # written under a private name and renamed: ranks of one box that generate the same file concurrently
    # (bench.py --gpus N --sites .. --taxa ..) never read a partial one
    tmp = "%s.%d.tmp" % (out, os.getpid())
    with open(tmp, "w") as fh:
        fh.write(txt)
    os.replace(tmp, out)
    return hashlib.sha256(txt.encode()).hexdigest()


if __name__ == "__main__":
    N, M, seed, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    print(write(N, M, seed, out))
