"""Drop-in overlay: run the reference's own scripts (train_v6.py, train_v5.py, test.py, test_vivo.py)
unchanged on the MI355X path by prepending this directory to PYTHONPATH:

    PYTHONPATH=/path/to/repo/dropin python train_v6.py --cfg ... --obj_name ape

The reference scripts put their own directory first on sys.path (``sys.path.insert(0, os.getcwd())``,
train_v6.py:9, test.py:12), so a plain PYTHONPATH entry would lose to the reference's own
``model/`` and ``common_ops.py``.  Python imports ``sitecustomize`` at start-up from the first
sys.path entry holding one; this one installs a meta-path finder ahead of the path scan that maps
exactly the hot-path modules to the overlay files next to it (each re-exports zebrapose_amd):

    model.BinaryCodeNet, model.BinaryCodeNet_v3     (train_v6.py:26-27, test.py:30, train_v5.py:26)
    binary_code_helper.CNN_output_to_pose           (train_v6.py:22, test.py:26)
    binary_code_helper.generate_new_dict            (test.py:38)
    common_ops, utils_v2, metric                    (train_v6.py:31, 35; test.py:32-35)

Every other module of the two packages (model.BinaryCodeNet_v2, binary_code_helper.
class_id_encoder_decoder, ...) still resolves to the reference's file, and every other top-level
module (config_parser, bop_dataset_pytorch, tools_for_BOP, ...) is untouched.  A sitecustomize
further down sys.path (site-packages, a harness hook) is executed afterwards, as Python would have.
"""
import importlib.abc
import importlib.util
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
_PACKAGES = ("model", "binary_code_helper")
_MODULES = {
    "model.BinaryCodeNet": "model/BinaryCodeNet.py",
    "model.BinaryCodeNet_v3": "model/BinaryCodeNet_v3.py",
    "binary_code_helper.CNN_output_to_pose": "binary_code_helper/CNN_output_to_pose.py",
    "binary_code_helper.generate_new_dict": "binary_code_helper/generate_new_dict.py",
    "common_ops": "common_ops.py",
    "utils_v2": "utils_v2.py",
    "metric": "metric.py",
}


class _OverlayFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, name, path=None, target=None):
        if name in _MODULES:
            return importlib.util.spec_from_file_location(name, os.path.join(_HERE, _MODULES[name]))
        if name in _PACKAGES:
            # the overlay package first, then every same-named package directory on sys.path (the
            # reference's), so the modules the overlay does not replace still import from there
            locs = [os.path.join(_HERE, name)]
            for entry in sys.path:
                d = os.path.join(os.path.abspath(entry or os.getcwd()), name)
                if d not in locs and os.path.isdir(d):
                    locs.append(d)
            return importlib.util.spec_from_file_location(name, os.path.join(_HERE, name, "__init__.py"),
                                                          submodule_search_locations=locs)
        return None


if not any(isinstance(f, _OverlayFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _OverlayFinder())
if _ROOT not in sys.path:
    sys.path.append(_ROOT)  # zebrapose_amd, after everything the reference expects


def _chain():
    """Run the sitecustomize Python would have imported had this one not been first."""
    for entry in sys.path:
        d = os.path.abspath(entry or os.getcwd())
        if d == _HERE:
            continue
        f = os.path.join(d, "sitecustomize.py")
        if os.path.isfile(f):
            spec = importlib.util.spec_from_file_location("_zp_chained_sitecustomize", f)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            return


_chain()
