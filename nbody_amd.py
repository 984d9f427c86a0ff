"""Import alias for the package directory
``extending-the-n-body-benchmark-a-cross-model-study-of-geometric-deep-learning-architectures_amd``
(not a valid identifier).  ``import nbody_amd`` registers it as the package
``nbody_amd`` so that ``nbody_amd.segnn`` etc. resolve normally."""
import importlib.util
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                       "extending-the-n-body-benchmark-a-cross-model-study-of-geometric-deep-learning-architectures_amd")

_spec = importlib.util.spec_from_file_location(__name__, os.path.join(PKG_DIR, "__init__.py"),
                                               submodule_search_locations=[PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
