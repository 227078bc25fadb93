"""Import shim: exposes the package directory `semi-direct-visual-odometry_amd/` (not a valid Python
identifier) as the importable module `svo_amd`."""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "semi-direct-visual-odometry_amd")
_spec = importlib.util.spec_from_file_location("svo_amd", os.path.join(_DIR, "__init__.py"),
                                              submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["svo_amd"] = _mod
_spec.loader.exec_module(_mod)
