"""Import shim for the ``tensorflow2-machine-vision_amd/`` package.

The package directory name required by the project layout contains hyphens and
so cannot be imported with a plain ``import`` statement.  Importing this module
loads that directory as the package ``tf2mv_amd`` and replaces this shim in
``sys.modules`` with it, so ``import tf2mv_amd`` and
``from tf2mv_amd.model import EfficientDetNetTrain`` work everywhere.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "tensorflow2-machine-vision_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_PKG_DIR, "__init__.py"),
    submodule_search_locations=[_PKG_DIR])
_pkg = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _pkg
_spec.loader.exec_module(_pkg)
