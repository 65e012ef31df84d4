"""Every module of the package, bench.py and the graft entry import on a CPU-only host (no GPU
call at import time), so a syntax or import error shows up in the CPU suite."""
import importlib
import pkgutil

import pytest

import loner_amd


@pytest.mark.parametrize("name", sorted(m.name for m in pkgutil.iter_modules(loner_amd.__path__)))
def test_package_module_imports(name):
    importlib.import_module(f"loner_amd.{name}")


@pytest.mark.parametrize("name", ["bench", "__graft_entry__"])
def test_top_level_imports(name):
    importlib.import_module(name)
