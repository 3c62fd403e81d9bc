"""Import helper: the package directory is ``dynamicfactormodels.jl_amd/`` (a
dot in the name, so it cannot be imported by name).  ``load()`` registers it
as the module ``dfm_amd``."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "dynamicfactormodels.jl_amd")


def load():
    if "dfm_amd" in sys.modules:
        return sys.modules["dfm_amd"]
    spec = importlib.util.spec_from_file_location(
        "dfm_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["dfm_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
