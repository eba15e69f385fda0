"""``binary_code_helper.CNN_output_to_pose`` -> zebrapose_amd (device decode + device RANSAC-EPnP)."""
from zebrapose_amd.binary_code_helper.CNN_output_to_pose import *  # noqa: F401,F403
from zebrapose_amd.binary_code_helper.CNN_output_to_pose import (CNN_outputs_to_object_pose,  # noqa: F401
                                                                 load_dict_class_id_3D_points)
