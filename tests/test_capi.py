"""The C-ABI library loads and exports every symbol include/loner_amd.h declares; host-only entry
points agree with the oracle.  CPU only (no kernel launches)."""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle import hashgrid as ohg
from oracle import rng as orng

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "loner_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lnr_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def L():
    from loner_amd import _lib
    return _lib


def test_library_exports_header(L):
    lib = L.lib()
    declared = _declared()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in include/loner_amd.h but not exported"
    assert set(declared) == set(L.exported_symbols()), set(declared) ^ set(L.exported_symbols())
    assert lib.lnr_version() == 1


def test_grid_desc_matches_tcnn_layout(L):
    for log2 in (18, 19):
        d = L.grid_desc(16, 2, log2, 16, 2.0)
        o = ohg.GridLayout(16, 2, log2, 16)
        assert d.n_entries == o.n_entries
        assert list(d.size[:16]) == o.sizes
        assert list(d.offset[:16]) == o.offsets
        assert list(d.resolution[:16]) == o.resolutions
        np.testing.assert_array_equal(np.array(d.scale[:16], np.float32), np.array(o.scales, np.float32))


def test_step_key_matches_oracle(L):
    for seed, step in [(0, 0), (1, 7), (123456, 99999)]:
        assert L.step_key(seed, step) == orng.step_key(seed, step)


def test_error_contract(L):
    d = L.GridDesc()
    rc = L.lib().lnr_grid_desc_init(ctypes.byref(d), 16, 3, 18, 16, 2.0)
    assert rc == -1
    assert b"n_features_per_level=2" in L.lib().lnr_last_error()
    with pytest.raises(RuntimeError, match="n_levels"):
        L.grid_desc(0, 2, 18, 16)
