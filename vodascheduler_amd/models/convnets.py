"""Small/medium convnets of the reference workloads.

* ``vgg16_cifar``: ``applications.VGG16(weights=None, classes=10)`` at 32x32 (reference
  examples/py/tensorflow2/tensorflow2_keras_cifar_elastic.py:148-151; 33,638,218 params as
  counted in SURVEY.md §2.8: conv 14.7 M + FC 18.9 M).
* ``KerasMnistCNN``: Conv32-Conv64-MaxPool-Dense128-Dense10 (reference
  tensorflow2_keras_mnist_elastic.py:101-110; 1,199,882 params).
* ``TorchMnistNet``: the PyTorch elastic example's 2-conv Net (reference
  examples/py/pytorch/pytorch_mnist_elastic.py:80-96; 21,840 params).
* ``InceptionV3``: ``applications.InceptionV3(weights=None, include_top=True, classes=10)`` at
  75x75 for CIFAR (reference tensorflow2_keras_cifar_elastic.py:107-108,148,
  tf2-keras-cifar10-inceptionv3-elastic.yaml): the full Keras topology -- stem, mixed0-2 (A),
  mixed3 (B), mixed4-7 (C), mixed8 (D), mixed9-10 (E), global average pool, 2048 -> 10 head --
  with Keras' conv2d_bn (bias-free conv + BatchNormalization(scale=False, eps=1e-3) + ReLU).
  21,823,274 parameters counted the Keras way (weights + BN beta + moving mean/var).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from ..ops.batchnorm import FusedBatchNorm2d
from ..ops.conv_bias import Conv2dSepBias
from ..ops.pool import FusedMaxPool2d, max_pool2d


def _vgg_block(cin, cout, n):
    layers = []
    for i in range(n):
        # bias add + bias gradient on our column-sum kernel (hipGraph-safe; ops/conv_bias.py)
        layers += [Conv2dSepBias(cin if i == 0 else cout, cout, 3, padding=1), nn.ReLU(inplace=True)]
    layers.append(FusedMaxPool2d(2))
    return layers


class VGG16(nn.Module):
    def __init__(self, num_classes=10, input_size=32):
        super().__init__()
        self.features = nn.Sequential(*_vgg_block(3, 64, 2), *_vgg_block(64, 128, 2), *_vgg_block(128, 256, 3),
                                      *_vgg_block(256, 512, 3), *_vgg_block(512, 512, 3))
        s = input_size // 32
        self.classifier = nn.Sequential(nn.Flatten(), nn.Linear(512 * s * s, 4096), nn.ReLU(inplace=True),
                                        nn.Linear(4096, 4096), nn.ReLU(inplace=True), nn.Linear(4096, num_classes))

    def forward(self, x):
        return self.classifier(self.features(x))


def vgg16_cifar(num_classes=10):
    return VGG16(num_classes, 32)


class KerasMnistCNN(nn.Module):
    def __init__(self):
        super().__init__()
        self.c1 = nn.Conv2d(1, 32, 3)
        self.c2 = nn.Conv2d(32, 64, 3)
        self.fc1 = nn.Linear(64 * 12 * 12, 128)
        self.fc2 = nn.Linear(128, 10)

    def forward(self, x):
        x = F.relu(self.c1(x))
        x = F.max_pool2d(F.relu(self.c2(x)), 2)
        return self.fc2(F.relu(self.fc1(torch.flatten(x, 1))))


class TorchMnistNet(nn.Module):
    """The reference's PyTorch MNIST net (pytorch_mnist_elastic.py:80-96), dropout included:
    Dropout2d after conv2 and dropout(0.5) after fc1, active in training mode only.  The
    random masks are reproducible across resizes and restores because the trainer's elastic
    state carries the RNG state (runtime/elastic.py TorchState)."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 10, kernel_size=5)
        self.conv2 = nn.Conv2d(10, 20, kernel_size=5)
        self.conv2_drop = nn.Dropout2d()
        self.fc1 = nn.Linear(320, 50)
        self.fc2 = nn.Linear(50, 10)

    def forward(self, x):
        x = F.relu(F.max_pool2d(self.conv1(x), 2))
        x = F.relu(F.max_pool2d(self.conv2_drop(self.conv2(x)), 2))
        x = F.relu(self.fc1(x.view(-1, 320)))
        x = F.dropout(x, training=self.training)
        return F.log_softmax(self.fc2(x), dim=1)


# ----------------------------------------------------------------- InceptionV3 (Keras)
class BasicConv(nn.Module):
    """Keras ``conv2d_bn``: Conv2D(use_bias=False) -> BatchNormalization(scale=False) -> ReLU,
    the BN + ReLU as one fused HIP pass."""

    def __init__(self, cin, cout, **kw):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, bias=False, **kw)
        self.bn = FusedBatchNorm2d(cout, eps=0.001, momentum=0.01, relu=True, scale=False)

    def forward(self, x):
        return self.bn(self.conv(x))


def _avg3(x):
    # Keras AveragePooling2D((3, 3), strides=1, padding="same") averages over the valid
    # window only (count_include_pad=False)
    return F.avg_pool2d(x, 3, 1, 1, count_include_pad=False)


class InceptionA(nn.Module):
    """mixed0-2: 1x1 | 1x1-5x5 | 1x1-3x3-3x3 | avgpool-1x1."""

    def __init__(self, cin, pool):
        super().__init__()
        self.b1 = BasicConv(cin, 64, kernel_size=1)
        self.b5 = nn.Sequential(BasicConv(cin, 48, kernel_size=1), BasicConv(48, 64, kernel_size=5, padding=2))
        self.b3 = nn.Sequential(BasicConv(cin, 64, kernel_size=1), BasicConv(64, 96, kernel_size=3, padding=1),
                                BasicConv(96, 96, kernel_size=3, padding=1))
        self.bp = BasicConv(cin, pool, kernel_size=1)

    def forward(self, x):
        return torch.cat([self.b1(x), self.b5(x), self.b3(x), self.bp(_avg3(x))], 1)


class InceptionB(nn.Module):
    """mixed3 (grid reduction): 3x3/2 | 1x1-3x3-3x3/2 | maxpool/2."""

    def __init__(self, cin):
        super().__init__()
        self.b3 = BasicConv(cin, 384, kernel_size=3, stride=2)
        self.bd = nn.Sequential(BasicConv(cin, 64, kernel_size=1), BasicConv(64, 96, kernel_size=3, padding=1),
                                BasicConv(96, 96, kernel_size=3, stride=2))

    def forward(self, x):
        return torch.cat([self.b3(x), self.bd(x), max_pool2d(x, 3, 2)], 1)


class InceptionC(nn.Module):
    """mixed4-7: factorised 7x7 branches."""

    def __init__(self, cin, c7):
        super().__init__()
        self.b1 = BasicConv(cin, 192, kernel_size=1)
        self.b7 = nn.Sequential(BasicConv(cin, c7, kernel_size=1), BasicConv(c7, c7, kernel_size=(1, 7), padding=(0, 3)),
                                BasicConv(c7, 192, kernel_size=(7, 1), padding=(3, 0)))
        self.bd = nn.Sequential(BasicConv(cin, c7, kernel_size=1), BasicConv(c7, c7, kernel_size=(7, 1), padding=(3, 0)),
                                BasicConv(c7, c7, kernel_size=(1, 7), padding=(0, 3)),
                                BasicConv(c7, c7, kernel_size=(7, 1), padding=(3, 0)),
                                BasicConv(c7, 192, kernel_size=(1, 7), padding=(0, 3)))
        self.bp = BasicConv(cin, 192, kernel_size=1)

    def forward(self, x):
        return torch.cat([self.b1(x), self.b7(x), self.bd(x), self.bp(_avg3(x))], 1)


class InceptionD(nn.Module):
    """mixed8 (grid reduction): 1x1-3x3/2 | 1x1-1x7-7x1-3x3/2 | maxpool/2."""

    def __init__(self, cin):
        super().__init__()
        self.b3 = nn.Sequential(BasicConv(cin, 192, kernel_size=1), BasicConv(192, 320, kernel_size=3, stride=2))
        self.b7 = nn.Sequential(BasicConv(cin, 192, kernel_size=1),
                                BasicConv(192, 192, kernel_size=(1, 7), padding=(0, 3)),
                                BasicConv(192, 192, kernel_size=(7, 1), padding=(3, 0)),
                                BasicConv(192, 192, kernel_size=3, stride=2))

    def forward(self, x):
        return torch.cat([self.b3(x), self.b7(x), max_pool2d(x, 3, 2)], 1)


class InceptionE(nn.Module):
    """mixed9-10: 1x1 | 1x1-(1x3 | 3x1) | 1x1-3x3-(1x3 | 3x1) | avgpool-1x1."""

    def __init__(self, cin):
        super().__init__()
        self.b1 = BasicConv(cin, 320, kernel_size=1)
        self.b3 = BasicConv(cin, 384, kernel_size=1)
        self.b3a = BasicConv(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.b3b = BasicConv(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.bd = nn.Sequential(BasicConv(cin, 448, kernel_size=1), BasicConv(448, 384, kernel_size=3, padding=1))
        self.bda = BasicConv(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.bdb = BasicConv(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.bp = BasicConv(cin, 192, kernel_size=1)

    def forward(self, x):
        b3 = self.b3(x)
        bd = self.bd(x)
        return torch.cat([self.b1(x), self.b3a(b3), self.b3b(b3), self.bda(bd), self.bdb(bd), self.bp(_avg3(x))], 1)


class InceptionV3(nn.Module):
    """Keras ``applications.InceptionV3(include_top=True)``; 75x75 inputs give 7x7 after the
    stem, 3x3 after mixed3 and 1x1 after mixed8."""

    def __init__(self, num_classes=10):
        super().__init__()
        self.stem = nn.Sequential(BasicConv(3, 32, kernel_size=3, stride=2), BasicConv(32, 32, kernel_size=3),
                                  BasicConv(32, 64, kernel_size=3, padding=1), FusedMaxPool2d(3, 2),
                                  BasicConv(64, 80, kernel_size=1), BasicConv(80, 192, kernel_size=3),
                                  FusedMaxPool2d(3, 2))
        self.a = nn.Sequential(InceptionA(192, 32), InceptionA(256, 64), InceptionA(288, 64))
        self.b = InceptionB(288)
        self.c = nn.Sequential(InceptionC(768, 128), InceptionC(768, 160), InceptionC(768, 160), InceptionC(768, 192))
        self.d = InceptionD(768)
        self.e = nn.Sequential(InceptionE(1280), InceptionE(2048))
        self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        x = self.e(self.d(self.c(self.b(self.a(self.stem(x))))))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def keras_param_count(model: nn.Module) -> int:
    """Parameters counted as Keras' ``model.count_params()``: weights + BN moving statistics."""
    n = sum(p.numel() for p in model.parameters())
    for m in model.modules():
        if isinstance(m, nn.BatchNorm2d) and m.track_running_stats:
            n += m.running_mean.numel() + m.running_var.numel()
    return n
