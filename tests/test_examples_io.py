"""Replay-buffer files (Coach.py:144-170), no GPU: the reference's own pickle is
read by the whitelisting loader, written back in its format, and the native npz round-trips."""
import collections
import io
import pickle

import numpy as np
import pytest

from yacht_amd import examples_io as X
from yacht_amd.state import pack_many


def _expected(golden):
    g = golden("examples_ref_expected.npz")
    n = len(g["values"])
    pi = np.zeros((n, 3226))
    pi[g["pi_rows"], g["pi_cols"]] = g["pi_vals"]
    return g, pi


def _check(hist, g, pi):
    assert [len(it) for it in hist] == list(g["sizes"])
    flat = [e for it in hist for e in it]
    assert np.array_equal(pack_many([b for b, _, _ in flat]), g["states"])
    assert np.array_equal(np.array([p for _, p, _ in flat]), pi)
    assert np.array_equal(np.array([v for _, _, v in flat]), g["values"])


def test_reads_the_reference_pickle(golden):
    import os
    from conftest import REPO
    g, pi = _expected(golden)
    hist = X.load_reference_examples(os.path.join(REPO, "tests", "golden", "examples_ref.pkl"))
    _check(hist, g, pi)


def test_refuses_foreign_globals(tmp_path):
    p = tmp_path / "evil.examples"
    with open(p, "wb") as f:
        pickle.Pickler(f).dump([collections.OrderedDict()])  # any global outside the whitelist
    with pytest.raises(pickle.UnpicklingError):
        X.load_reference_examples(str(p))


def test_reference_format_round_trip(golden, tmp_path):
    import os
    from conftest import REPO
    g, pi = _expected(golden)
    hist = X.load_reference_examples(os.path.join(REPO, "tests", "golden", "examples_ref.pkl"))
    out = tmp_path / "ours.examples"
    X.save_reference_examples(str(out), hist)
    calls = []

    class Spy(pickle.Unpickler):  # what the reference's Unpickler would be asked to import
        def find_class(self, module, name):
            calls.append((module, name))
            return X._ReferenceUnpickler.find_class(self, module, name)

    with open(out, "rb") as f:
        back = Spy(f).load()
    assert set(calls) == {("collections", "deque"), ("yacht.YachtGame", "YachtState"),
                          ("yacht.YachtGame", "PlayerState")}
    assert all(isinstance(it, collections.deque) for it in back)
    _check(X.load_reference_examples(str(out)), g, pi)


def test_native_format_round_trip(golden, tmp_path):
    import os
    from conftest import REPO
    g, pi = _expected(golden)
    hist = X.load_reference_examples(os.path.join(REPO, "tests", "golden", "examples_ref.pkl"))
    p = str(tmp_path / "buf.npz")
    X.save_examples(p, hist)
    _check(X.load_examples(p), g, pi)
    s, t, v = X.to_device_arrays(X.load_examples(p))
    assert np.array_equal(s, g["states"]) and np.array_equal(t, pi.argmax(axis=1)) and len(v) == len(s)
