"""EDSR plugin: drop-in for sres/model/edsr/network.py (get_model :7-8, EDSR :9-32)."""
import torch.nn as nn

from ..common import SRNet


class EDSR(SRNet):
    arch = "edsr"


def get_model(**config) -> nn.Module:
    return EDSR(**config)
