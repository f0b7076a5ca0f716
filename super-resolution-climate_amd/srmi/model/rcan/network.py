"""RCAN plugin: drop-in for sres/model/rcan/network.py (get_model :5-6, RCAN :7-27).

Hyper-parameters come from cfg().model exactly as the reference's FModule
reads them (defaults cbottleneck=2, nblocks=20; common.py:9-28); the module's
state_dict keys and shapes equal the reference's.  Forward/backward run on the
srmi HIP engine (gfx950).
"""
import torch.nn as nn

from ..common import SRNet


class RCAN(SRNet):
    arch = "rcan"


def get_model(**config) -> nn.Module:
    return RCAN(**config)
