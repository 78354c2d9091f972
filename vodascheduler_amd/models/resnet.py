"""ResNet family (ResNet-50 v1.5 bottleneck) for the elastic training workloads.

Reference workload: ``applications.ResNet50(weights=None, classes=10)`` on CIFAR-10
(reference examples/py/tensorflow2/tensorflow2_keras_cifar_elastic.py:148-151) and the
BASELINE config "8 ResNet-50 ImageNet-shape jobs".  Convolutions run on MIOpen
through PyTorch-ROCm in channels_last bf16 (NHWC is MIOpen's fast layout on CDNA);
random-init weights, synthetic data.  Every BatchNorm is the fused HIP
BN(+residual)(+ReLU) of ops/batchnorm.py: the bottleneck's ``relu(bn3(conv3) + identity)``
is ONE statistics pass + ONE apply pass forward, instead of MIOpen BN + add + ReLU.  The 1x1
convolutions (with >= 128 input channels) run as GEMMs on the NHWC views with the split-K
MFMA weight-gradient kernel (ops/conv1x1.py); the 3x3 convolutions with >= 128 channels take
their weight gradient from the implicit-GEMM form of the same kernel (ops/conv3x3.py), and
the bottleneck's shortcut gradient is accumulated by conv1's input-gradient GEMM
(ops/conv1x1.GradSink).
"""
from __future__ import annotations

import os

import torch
from torch import nn

from ..ops.batchnorm import FusedBatchNorm2d
from ..ops.conv1x1 import USE_GRAD_SINK, Conv1x1, GradSink, fused_dgrad_bn_ok
from ..ops.conv3x3 import ConvKxK
from ..ops.pool import GlobalAvgPool2d
from ..ops.stem import FusedStem

# VODA_BN_PAIR=0: downsample blocks run bn3 and the shortcut BN as two fused BNs (A/B switch for
# ops/batchnorm._BNAct2Fn)
FUSE_DOWNSAMPLE_BN = os.environ.get("VODA_BN_PAIR", "1") != "0"


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None):
        super().__init__()
        width = planes
        self.conv1 = Conv1x1(inplanes, width)
        self.bn1 = FusedBatchNorm2d(width, relu=True)
        self.conv2 = ConvKxK(width, width, 3, stride=stride, padding=1)  # v1.5: stride on 3x3
        self.bn2 = FusedBatchNorm2d(width, relu=True)
        self.conv3 = Conv1x1(width, planes * self.expansion)
        self.bn3 = FusedBatchNorm2d(planes * self.expansion, relu=True)  # relu(bn3(.) + identity)
        self.downsample = downsample

    def forward(self, x):
        # x feeds conv1 and the shortcut: the shortcut's input gradient is handed to conv1's
        # input-gradient GEMM (beta = 1) instead of being added by autograd (ops/conv1x1.GradSink)
        sink = None
        if (USE_GRAD_SINK and self.training and torch.is_grad_enabled() and x.requires_grad
                and self.conv1._gemm_ok(x)):
            # identity blocks at fp32: conv1's input gradient reads bn3's masked shortcut
            # gradient in its epilogue (ops/conv1x1.fused_dgrad_bn), so bn3 hands it over unwritten
            lazy = (self.downsample is None and x.dtype == torch.float32 and self.conv1.stride == (1, 1)
                    and fused_dgrad_bn_ok(x.shape[0] * x.shape[2] * x.shape[3], self.conv1.in_channels,
                                          self.conv1.out_channels))
            sink = GradSink(lazy)
        out = self.bn1(self.conv1(x, sink_in=sink))
        out = self.bn2(self.conv2(out))
        if self.downsample is None:
            return self.bn3(self.conv3(out), x, sink=sink)
        ds = self.downsample
        if isinstance(ds, nn.Sequential) and len(ds) == 2 and isinstance(ds[0], Conv1x1):
            y_ds = ds[0](x, sink_out=sink)
            if FUSE_DOWNSAMPLE_BN and isinstance(ds[1], FusedBatchNorm2d):
                # relu(bn3(y3) + bn_ds(y_ds)) as one dual-BN op: the shortcut tensor is never
                # written, and one reduce + one apply pass give both BNs' gradients
                return self.bn3.forward_pair(self.conv3(out), ds[1], y_ds)
            idt = ds[1](y_ds)
        else:
            idt = ds(x)
        return self.bn3(self.conv3(out), idt)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None):
        super().__init__()
        self.conv1 = ConvKxK(inplanes, planes, 3, stride=stride, padding=1)
        self.bn1 = FusedBatchNorm2d(planes, relu=True)
        self.conv2 = ConvKxK(planes, planes, 3, padding=1)
        self.bn2 = FusedBatchNorm2d(planes, relu=True)  # relu(bn2(.) + identity)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        return self.bn2(self.conv2(self.bn1(self.conv1(x))), idt)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes: int = 1000, small_input: bool = False):
        super().__init__()
        self.inplanes = 64
        if small_input:  # CIFAR-style 32x32 stem
            self.stem = nn.Sequential(nn.Conv2d(3, 64, 3, padding=1, bias=False), FusedBatchNorm2d(64, relu=True))
        else:
            # conv 7x7/2 with the BN statistics in its epilogue, then BN + ReLU + 3x3/2 max
            # pool as one fused op (ops/stem.FusedStem); state dict keys stem.0.* / stem.1.*
            # as with a separate conv, BN and pool
            self.stem = FusedStem(3, 64)
        self.layer1 = self._make(block, 64, layers[0])
        self.layer2 = self._make(block, 128, layers[1], stride=2)
        self.layer3 = self._make(block, 256, layers[2], stride=2)
        self.layer4 = self._make(block, 512, layers[3], stride=2)
        self.pool = GlobalAvgPool2d()  # nn.AdaptiveAvgPool2d(1), channels_last HIP backward
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        for m in self.modules():  # zero-init last BN of each residual branch
            if isinstance(m, Bottleneck):
                nn.init.zeros_(m.bn3.weight)
            elif isinstance(m, BasicBlock):
                nn.init.zeros_(m.bn2.weight)

    def _make(self, block, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(Conv1x1(self.inplanes, planes * block.expansion, stride=stride),
                                 FusedBatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.stem(x)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.pool(x), 1))


def resnet50(num_classes: int = 1000, small_input: bool = False) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, small_input)


def resnet18(num_classes: int = 1000, small_input: bool = False) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, small_input)
