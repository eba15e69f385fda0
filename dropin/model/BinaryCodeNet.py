"""``model.BinaryCodeNet`` (reference model/BinaryCodeNet.py) -> zebrapose_amd, HIP-executed."""
from zebrapose_amd.model.BinaryCodeNet import *  # noqa: F401,F403
from zebrapose_amd.model.BinaryCodeNet import (BinaryCodeLoss, BinaryCodeNet_Deeplab, BinaryLossWeighted,  # noqa: F401
                                               DeepLabV3, HammingLoss, MaskLoss)
