"""``metric`` (reference metric.py) -> zebrapose_amd (device ADD / ADI)."""
from zebrapose_amd.metric import *  # noqa: F401,F403
from zebrapose_amd.metric import Calculate_ADD_Error_BOP, Calculate_ADI_Error_BOP  # noqa: F401
