"""Regression test for the train-mode BN statistics buffer (fixed overrun, commit d97ffd1): the
caller sizes the per-launch partials with zp_conv2d_stat_parts, and zp_conv2d now refuses a launch
whose grid would emit a different number of parts.  Every tile override the dispatch honours
(ZP_CONV_TP=128|256, ZP_CONV_TC256=0, ZP_CONV_STRIP=0, the 256-channel tile forced on every
eligible layer through zp_conv_tuning, and the combination that overran: the 256-channel tile plus
a 128-pixel override) runs one bf16 train-mode forward of the network (every conv with BN emits
statistics) in its own process (the overrides are read once per process).  Each must succeed and
land near the default configuration's logits (different tiles change only f32 accumulation order)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import json, os, sys
sys.path.insert(0, os.environ["ZP_ROOT"])
import numpy as np, torch
import zebrapose_amd._lib as L
from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
if os.environ.get("FORCE256") == "1":
    L.lib.zp_conv_tuning(0, 1)
torch.manual_seed(0)
net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="bf16").cuda().train()
g = torch.Generator().manual_seed(3)
x = torch.randn(4, 3, 128, 128, generator=g).cuda()
with torch.no_grad():
    m, c = net(x)
torch.cuda.synchronize()
rm = float(net.net.aspp.upsample_2[7].running_mean.double().sum())
print(json.dumps({"mask": m.cpu().numpy().ravel()[::97].tolist(), "code": c.cpu().numpy().ravel()[::97].tolist(),
                  "rm": rm}))
"""

CONFIGS = {
    "default": {},
    "tp128": {"ZP_CONV_TP": "128"},
    "tp256": {"ZP_CONV_TP": "256"},
    "no_tc256": {"ZP_CONV_TC256": "0"},
    "no_strip": {"ZP_CONV_STRIP": "0"},
    "force_tc256": {"FORCE256": "1"},
    "force_tc256_tp128": {"FORCE256": "1", "ZP_CONV_TP": "128", "ZP_CONV_STRIP": "0"},
}


def test_stat_parts_match_launch_under_every_override(gpu):
    out = {}
    for name, extra in CONFIGS.items():
        env = dict(os.environ, ZP_ROOT=ROOT, ZP_QUIET="1", **extra)
        r = subprocess.run([sys.executable, "-c", SCRIPT], capture_output=True, text=True, timeout=180, env=env,
                           cwd=ROOT)
        assert r.returncode == 0, (name, r.stderr[-3000:])
        out[name] = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    base = out["default"]
    for name, rec in out.items():
        for k in ("mask", "code"):
            a, b = np.asarray(rec[k]), np.asarray(base[k])
            assert np.isfinite(a).all(), name
            rel = np.linalg.norm(a - b) / np.linalg.norm(b)
            print(f"{name}: {k} rel-L2 vs default {rel:.4f}")
            assert rel <= 0.3, (name, k, rel)
        assert abs(rec["rm"] - base["rm"]) <= 0.05 * abs(base["rm"]) + 1e-3, (name, rec["rm"], base["rm"])
