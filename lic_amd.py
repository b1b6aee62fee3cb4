"""Import shim: exposes the package directory
`learning-driven-image-compression-algorithm_amd/` (not a valid Python
identifier) under the importable name ``lic_amd``.

``import lic_amd`` (with the repo root on ``sys.path``) loads the package's
``__init__.py`` and registers it in ``sys.modules`` so that ``lic_amd.model``
etc. resolve through the package ``__path__``.
"""
import importlib.util
import pathlib
import sys

_PKG_DIR = pathlib.Path(__file__).resolve().parent / "learning-driven-image-compression-algorithm_amd"
_spec = importlib.util.spec_from_file_location(
    __name__, _PKG_DIR / "__init__.py", submodule_search_locations=[str(_PKG_DIR)])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
