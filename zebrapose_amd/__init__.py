"""zebrapose_amd -- MI355X (gfx950) implementation of ZebraPose's data-parallel hot path.

Drop-in modules mirror the reference package layout:
  zebrapose_amd.model.BinaryCodeNet      BinaryCodeNet_Deeplab, BinaryCodeLoss, MaskLoss, ...
  zebrapose_amd.common_ops               from_output_to_class_mask / _binary_code, get_batch_size
  zebrapose_amd.binary_code_helper       code -> vertex decode (device), LUT loading
  zebrapose_amd.utils_v2                 checkpoint save / load (reference layout)
The arithmetic lives in libzp.so (include/zp.h), loaded by zebrapose_amd._lib.
"""
__version__ = "0.1.0"
