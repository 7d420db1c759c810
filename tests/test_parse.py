"""Dataset parser (sr_parse_dataset) against the oracle's mcmc_readmodel restatement.

mcmc.c:339-437: header "N M" read with fgets(MAXS); each site row read with one
fgets(MAXS) call; characters other than '0'/'1' are skipped; a '*' after the M-th digit
marks a hard site.  A row longer than MAXS-1 characters is therefore split, exactly as
in the reference (maxs=0 lifts the limit -- SURVEY.md §8f-4).
"""
import os

import numpy as np
import pytest

import oracle_ref
import seriation_amd as sa
from seriation_amd import _lib as L

HERE = os.path.dirname(os.path.abspath(__file__))
DS = os.path.join(HERE, "golden", "datasets")
NAMES = sorted(os.listdir(DS))


def _read(name):
    with open(os.path.join(DS, name), "rb") as fh:
        return fh.read()


def _same(text, maxs):
    rc, X, h = oracle_ref.parse(text, maxs)
    assert rc == 0
    ds = sa.Dataset.parse(text, maxs)
    np.testing.assert_array_equal(ds.X, X.astype(np.uint8))
    np.testing.assert_array_equal(ds.hard, h.astype(np.uint8))
    assert ds.nh == int(h.sum())
    return ds


@pytest.mark.parametrize("name", NAMES)
def test_reference_datasets(name):
    ds = _same(_read(name), 2000)
    expect = {"g2s2.txt": (526, 296, 15), "g10s10.txt": (124, 139, 11), "synth_256x512.txt": (256, 512, 12)}
    if name in expect:
        assert (ds.N, ds.M, ds.nh) == expect[name]


def test_skips_other_characters_and_marks_hard():
    text = b"3 4\n1,0;1 x 1 *\n0 0 0 1\n1 1 1 1*\n"
    ds = _same(text, 2000)
    assert ds.X.tolist() == [[1, 0, 1, 1], [0, 0, 0, 1], [1, 1, 1, 1]]
    assert ds.hard.tolist() == [1, 0, 1]


def test_long_rows_split_like_fgets():
    rng = np.random.default_rng(3)
    N, M = 6, 1500                      # 3000-char rows > MAXS-1
    X = (rng.random((N, M)) < 0.3).astype(int)
    rows = [" ".join(map(str, r)) + (" *" if i == 2 else "") for i, r in enumerate(X)]
    text = ("%d %d\n" % (N, M) + "\n".join(rows) + "\n").encode()
    ds = _same(text, 0)                 # unlimited lines: the matrix as written
    np.testing.assert_array_equal(ds.X, X)
    _same(text, 2000)                   # reference limit: rows split exactly as fgets does
    _same(text, 17)


@pytest.mark.parametrize("text,code", [
    (b"", L.SR_EPARSE),
    (b"abc\n", L.SR_EHEADER),
    (b"0 5\n", L.SR_EHEADER),
    (b"3 2\n1 0\n", L.SR_EPARSE),
])
def test_errors(text, code):
    with pytest.raises(sa.SrError) as e:
        sa.Dataset.parse(text)
    assert e.value.code == code
    rc, _, _ = oracle_ref.parse(text) if text else (-2, None, None)
    assert rc != 0


def test_load_missing_file():
    with pytest.raises(sa.SrError) as e:
        sa.Dataset.load("/nonexistent/dataset.txt")
    assert e.value.code == L.SR_EIO


def test_binary_bitpacked_roundtrip(tmp_path, datasets_dir):
    """sr_save_dataset_bin / sr_load_dataset_bin (SURVEY §8f-4 extension): exact round trip of X
    and the hard flags, ~32x smaller than the text, and sr_load_dataset recognises the magic."""
    import seriation_amd as sa
    for name in ("g10s10.txt", "g2s2.txt", "synth_256x512.txt"):
        src = os.path.join(datasets_dir, name)
        ds = sa.Dataset.load(src)
        p = str(tmp_path / (name + ".srb"))
        ds.save_bin(p)
        for back in (sa.Dataset.load_bin(p), sa.Dataset.load(p)):
            assert (back.N, back.M, back.nh) == (ds.N, ds.M, ds.nh)
            assert np.array_equal(back.X, ds.X) and np.array_equal(back.hard, ds.hard)
        assert os.path.getsize(p) * 8 < os.path.getsize(src) * 1.2
    # odd widths and a corrupt header
    X = (np.arange(7 * 13).reshape(7, 13) % 3 == 0).astype(np.uint8)
    ds = sa.Dataset(X, np.array([0, 1, 0, 0, 1, 0, 0], bool))
    p = str(tmp_path / "odd.srb")
    ds.save_bin(p)
    back = sa.Dataset.load_bin(p)
    assert np.array_equal(back.X, X) and back.nh == 2
    with open(p, "r+b") as fh:
        fh.seek(4)
        fh.write(b"\x07\x00\x00\x00")
    with pytest.raises(sa.SrError):
        sa.Dataset.load_bin(p)
