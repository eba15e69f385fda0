"""``common_ops`` (reference common_ops.py) -> zebrapose_amd (device threshold)."""
from zebrapose_amd.common_ops import *  # noqa: F401,F403
from zebrapose_amd.common_ops import (from_output_to_class_binary_code, from_output_to_class_mask,  # noqa: F401
                                      get_batch_size)
