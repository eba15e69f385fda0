"""``model.BinaryCodeNet_v3`` (reference model/BinaryCodeNet_v3.py) -> zebrapose_amd."""
from zebrapose_amd.model.BinaryCodeNet_v3 import *  # noqa: F401,F403
from zebrapose_amd.model.BinaryCodeNet_v3 import BinaryCodeNet_Deeplab_v3  # noqa: F401

