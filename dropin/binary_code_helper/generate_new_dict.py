"""``binary_code_helper.generate_new_dict`` -> zebrapose_amd (device LUT coarsening)."""
from zebrapose_amd.binary_code_helper.generate_new_dict import *  # noqa: F401,F403
from zebrapose_amd.binary_code_helper.generate_new_dict import generate_new_corres_dict  # noqa: F401
