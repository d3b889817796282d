"""Import shim: ``import pcm_amd`` loads the package directory
``3d-point-cloud-multiday-imagery_amd/`` (not a valid Python identifier)."""
import importlib.util as _u
import os as _os
import sys as _sys

_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "3d-point-cloud-multiday-imagery_amd")
_spec = _u.spec_from_file_location(__name__, _os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR])
_mod = _u.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
