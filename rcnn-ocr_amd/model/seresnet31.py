"""SE-ResNet31 parameter tree with the reference's module names.

Mirrors model/seresnet31.py of sherstpasha/RCNN-OCR (SELayer :5-20, SEBasicBlock
:23-67, SEResNet31 :70-187) so state_dicts are interchangeable. Compute does
not run through these torch modules: RCNN.encode/forward dispatch the whole
backbone to the HIP engine (crnn_hip.engine), which reads these parameters.
"""
from __future__ import annotations

import torch.nn as nn


class SELayer(nn.Module):
    """squeeze-excitation: fc = Linear(C, C/r, no bias) -> ReLU -> Linear(C/r, C, no bias) -> Sigmoid."""

    def __init__(self, channel, reduction=16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        hidden = channel // reduction
        self.fc = nn.Sequential(nn.Linear(channel, hidden, bias=False), nn.ReLU(inplace=True),
                                nn.Linear(hidden, channel, bias=False), nn.Sigmoid())

    def forward(self, x):
        raise NotImplementedError("SE blocks run inside the HIP engine; call RCNN.encode/forward")


class DropBlock2d(nn.Module):
    """torchvision.ops.DropBlock2d's attributes (p, block_size, inplace, eps) as SEBasicBlock holds
    it (model/seresnet31.py:49-53). Parameter-free; in training the mask is drawn and applied inside
    the HIP engine (crnn_dropblock_mask / crnn_se_residual_drop_fwd), identity in eval."""

    def __init__(self, p: float, block_size: int, inplace: bool = False, eps: float = 1e-6):
        super().__init__()
        self.p, self.block_size, self.inplace, self.eps = p, block_size, inplace, eps

    def forward(self, x):
        raise NotImplementedError("DropBlock2d runs inside the HIP engine; call RCNN.encode/forward")

    def extra_repr(self):
        return f"p={self.p}, block_size={self.block_size}, inplace={self.inplace}"


class SEBasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, reduction=16, dropblock_p=0.0,
                 dropblock_block_size=5):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.se = SELayer(planes, reduction)
        self.downsample = downsample
        self.dropblock = DropBlock2d(p=dropblock_p, block_size=dropblock_block_size) if dropblock_p > 0 \
            else nn.Identity()
        self.stride = stride

    def forward(self, x):
        raise NotImplementedError("SE blocks run inside the HIP engine; call RCNN.encode/forward")


class SEResNet31(nn.Module):
    """stem (2 x conv3x3+BN+ReLU, maxpool) -> stages of 1/2/5/3 SE blocks -> conv_out (2 x conv2x2+BN+ReLU)."""

    STAGES = (("layer1", 128, 256, 1, 2), ("layer2", 256, 256, 2, 1),
              ("layer3", 256, 512, 5, 2), ("layer4", 512, 512, 3, 1))

    def __init__(self, in_channels=3, out_channels=512, reduction=16, dropblock_p=0.0, dropblock_block_size=5):
        super().__init__()
        if in_channels != 3 or out_channels != 512:
            raise NotImplementedError("the HIP backbone is built for 3 -> 512 channels (reference defaults)")
        self.conv0 = nn.Sequential(
            nn.Conv2d(in_channels, 64, 3, 1, 1, bias=False), nn.BatchNorm2d(64), nn.ReLU(True),
            nn.Conv2d(64, 128, 3, 1, 1, bias=False), nn.BatchNorm2d(128), nn.ReLU(True),
            nn.MaxPool2d(2, 2))
        for name, inp, planes, blocks, stride in self.STAGES:
            setattr(self, name, self._make_layer(inp, planes, blocks, stride, reduction, dropblock_p,
                                                 dropblock_block_size))
        self.conv_out = nn.Sequential(
            nn.Conv2d(512, out_channels, 2, stride=(2, 1), padding=(0, 1), bias=False),
            nn.BatchNorm2d(out_channels), nn.ReLU(True),
            nn.Conv2d(out_channels, out_channels, 2, stride=1, padding=0, bias=False),
            nn.BatchNorm2d(out_channels), nn.ReLU(True))
        self.out_channels = out_channels

    @staticmethod
    def _make_layer(inplanes, planes, blocks, stride, reduction, dropblock_p, dropblock_block_size):
        ds = None
        if stride != 1 or inplanes != planes:
            ds = nn.Sequential(nn.Conv2d(inplanes, planes, 1, stride=stride, bias=False), nn.BatchNorm2d(planes))
        layers = [SEBasicBlock(inplanes, planes, stride, ds, reduction, dropblock_p, dropblock_block_size)]
        layers += [SEBasicBlock(planes, planes, 1, None, reduction, dropblock_p, dropblock_block_size)
                   for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        raise NotImplementedError("the backbone runs inside the HIP engine; call RCNN.encode/forward")
