"""The drop-in overlay (dropin/): the reference scripts' own import lines -- train_v6.py:22-35,
train_v5.py:22-36, test.py:26-43 -- executed verbatim under ``PYTHONPATH=dropin`` from a working
directory that holds the reference's module names (the scripts run ``sys.path.insert(0,
os.getcwd())`` first, train_v6.py:9 / test.py:12, so the cwd copies would normally win).  Stubs
stand in for the reference's files here (they raise if imported); the hot-path modules must come
from zebrapose_amd and every other module of those packages must still come from the cwd."""
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

REFERENCE_IMPORTS = """
import os, sys
sys.path.insert(0, os.getcwd())
from binary_code_helper.CNN_output_to_pose import load_dict_class_id_3D_points
from model.BinaryCodeNet import BinaryCodeNet_Deeplab
from model.BinaryCodeNet import MaskLoss, BinaryCodeLoss
from utils_v2 import save_checkpoint, get_checkpoint
from common_ops import from_output_to_class_mask, get_batch_size
from binary_code_helper.CNN_output_to_pose import load_dict_class_id_3D_points, CNN_outputs_to_object_pose
from model.BinaryCodeNet_v3 import BinaryCodeNet_Deeplab_v3
from utils_v2 import save_checkpoint, get_checkpoint, save_best_checkpoint
from metric import Calculate_ADD_Error_BOP, Calculate_ADI_Error_BOP
from common_ops import from_output_to_class_mask, from_output_to_class_binary_code, get_batch_size
from binary_code_helper.generate_new_dict import generate_new_corres_dict
from binary_code_helper.class_id_encoder_decoder import RGB_image_to_class_id_image
from model.BinaryCodeNet_v2 import MARK as V2
import config_parser
import json
mods = {n: getattr(sys.modules[n], "__file__", "") for n in (
    "model.BinaryCodeNet", "model.BinaryCodeNet_v3", "binary_code_helper.CNN_output_to_pose",
    "binary_code_helper.generate_new_dict", "common_ops", "utils_v2", "metric",
    "binary_code_helper.class_id_encoder_decoder", "model.BinaryCodeNet_v2", "config_parser")}
print(json.dumps({"files": mods, "net": BinaryCodeNet_Deeplab.__module__, "loss": BinaryCodeLoss.__module__,
                  "v2": V2, "cid": RGB_image_to_class_id_image(None)}))
"""

RAISE = "raise ImportError('the reference copy was imported instead of the overlay')\n"


def _fake_reference(d):
    """The reference's module names in a directory, as the scripts' cwd."""
    for rel in ("model/BinaryCodeNet.py", "model/BinaryCodeNet_v3.py", "binary_code_helper/CNN_output_to_pose.py",
                "binary_code_helper/generate_new_dict.py", "common_ops.py", "utils_v2.py", "metric.py"):
        p = os.path.join(d, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(RAISE)
    for pkg in ("model", "binary_code_helper"):
        with open(os.path.join(d, pkg, "__init__.py"), "w") as f:
            f.write("")
    with open(os.path.join(d, "model", "BinaryCodeNet_v2.py"), "w") as f:
        f.write("MARK = 'reference v2'\n")
    with open(os.path.join(d, "binary_code_helper", "class_id_encoder_decoder.py"), "w") as f:
        f.write("def RGB_image_to_class_id_image(x):\n    return 'reference encoder'\n")
    with open(os.path.join(d, "config_parser.py"), "w") as f:
        f.write("def parse_cfg(p):\n    return {}\n")


def test_reference_import_lines_resolve_to_overlay(tmp_path):
    _fake_reference(str(tmp_path))
    script = tmp_path / "train_like.py"
    script.write_text(textwrap.dedent(REFERENCE_IMPORTS))
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "dropin"), ZP_QUIET="1")
    r = subprocess.run([sys.executable, str(script)], cwd=str(tmp_path), env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    files = out["files"]
    for n in ("model.BinaryCodeNet", "model.BinaryCodeNet_v3", "binary_code_helper.CNN_output_to_pose",
              "binary_code_helper.generate_new_dict", "common_ops", "utils_v2", "metric"):
        assert files[n].startswith(os.path.join(ROOT, "dropin")), (n, files[n])
    assert out["net"] == "zebrapose_amd.model.BinaryCodeNet" and out["loss"] == "zebrapose_amd.model.BinaryCodeNet"
    # everything the overlay does not replace still comes from the reference's directory
    for n in ("binary_code_helper.class_id_encoder_decoder", "model.BinaryCodeNet_v2", "config_parser"):
        assert files[n].startswith(str(tmp_path)), (n, files[n])
    assert out["v2"] == "reference v2" and out["cid"] == "reference encoder"
