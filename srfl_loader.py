"""Import shim for the product package.

The package lives in ``secure-robust-federated-learning_amd/`` (the name the
build contract fixes), which is not a valid Python identifier.  ``load()``
registers it in ``sys.modules`` as ``srfl_amd`` so that ``import srfl_amd`` and
``from srfl_amd import robust_estimator`` work everywhere (tests, bench,
``__graft_entry__``, and a reference checkout that wants the drop-in module).
"""
from __future__ import annotations

import importlib.util
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "secure-robust-federated-learning_amd")
NAME = "srfl_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
