"""``utils_v2`` (reference utils_v2.py) -> zebrapose_amd (same checkpoint layout)."""
from zebrapose_amd.utils_v2 import *  # noqa: F401,F403
from zebrapose_amd.utils_v2 import get_checkpoint, save_best_checkpoint, save_checkpoint  # noqa: F401
