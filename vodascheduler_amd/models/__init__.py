"""Model zoo + synthetic-data workload registry.

Every workload of the reference (W1 ResNet50/VGG16/InceptionV3 on CIFAR-10,
W2 Keras MNIST CNN, W3 Transformer NMT, W4 PyTorch MNIST) plus the BASELINE configs'
ResNet-50 ImageNet-shape and BERT-base, with random-init weights and synthetic batches of the
real shapes (no datasets are available offline).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable

import torch
import torch.nn.functional as F

from .convnets import InceptionV3, KerasMnistCNN, TorchMnistNet, vgg16_cifar
from .resnet import resnet18, resnet50
from .transformer import BertBase, TransformerNMT


@dataclass
class Workload:
    name: str
    build: Callable[[], torch.nn.Module]
    make_batch: Callable[[int, torch.device, torch.Generator | None], tuple]
    loss: Callable[[torch.nn.Module, tuple], torch.Tensor]
    per_gpu_batch: int
    optimizer: str = "sgd"
    opt_kwargs: dict = field(default_factory=dict)
    channels_last: bool = False
    samples_unit: str = "img"   # throughput unit (img or tok)
    tokens_per_sample: int = 1


def _img_batch(c, h, w, classes):
    def mk(b, dev, g=None):
        x = torch.randn(b, c, h, w, device=dev, generator=g)
        y = torch.randint(0, classes, (b,), device=dev, generator=g)
        return x, y
    return mk


def _ce(model, batch):
    x, y = batch
    return F.cross_entropy(model(x).float(), y)


def _nll(model, batch):
    x, y = batch
    return F.nll_loss(model(x).float(), y)


def _nmt_batch(b, dev, g=None, vocab=15000, T=20):
    src = torch.randint(1, vocab, (b, T), device=dev, generator=g)
    tgt = torch.randint(1, vocab, (b, T + 1), device=dev, generator=g)
    src[:, -3:] = 0  # some padding, as in the reference's padded sentences
    return src, tgt[:, :-1], tgt[:, 1:]


def _nmt_loss(model, batch):
    src, tin, tout = batch
    logits = model(src, tin)
    return F.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), tout.reshape(-1), ignore_index=0)


def _bert_batch(b, dev, g=None, vocab=30522, T=128):
    ids = torch.randint(1000, vocab, (b, T), device=dev, generator=g)
    mask = torch.ones(b, T, device=dev, dtype=torch.bool)
    labels = torch.full((b, T), -100, device=dev, dtype=torch.long)
    sel = torch.rand(b, T, device=dev, generator=g) < 0.15
    labels[sel] = ids[sel]
    return ids, mask, labels


def _bert_loss(model, batch):
    ids, mask, labels = batch
    logits = model(ids, mask)
    return F.cross_entropy(logits.float().view(-1, logits.shape[-1]), labels.view(-1), ignore_index=-100)


WORKLOADS: dict[str, Workload] = {
    "resnet50": Workload("resnet50", lambda: resnet50(1000), _img_batch(3, 224, 224, 1000), _ce, 256, "sgd",
                         dict(lr=0.1, momentum=0.9, weight_decay=5e-5), channels_last=True),
    "resnet50-cifar": Workload("resnet50-cifar", lambda: resnet50(10, small_input=True), _img_batch(3, 32, 32, 10),
                               _ce, 128, "sgd", dict(lr=0.01, momentum=0.9), channels_last=True),
    "resnet18": Workload("resnet18", lambda: resnet18(1000), _img_batch(3, 224, 224, 1000), _ce, 256, "sgd",
                         dict(lr=0.1, momentum=0.9), channels_last=True),
    "vgg16": Workload("vgg16", vgg16_cifar, _img_batch(3, 32, 32, 10), _ce, 128, "sgd",
                      dict(lr=0.01, momentum=0.9), channels_last=True),
    "inceptionv3": Workload("inceptionv3", InceptionV3, _img_batch(3, 75, 75, 10), _ce, 128, "rmsprop",
                            dict(lr=1e-3), channels_last=True),
    "mnist": Workload("mnist", KerasMnistCNN, _img_batch(1, 28, 28, 10), _ce, 128, "adam", dict(lr=1e-3)),
    "mnist-torch": Workload("mnist-torch", TorchMnistNet, _img_batch(1, 28, 28, 10), _nll, 64, "sgd",
                            dict(lr=0.01, momentum=0.5)),
    "transformer": Workload("transformer", TransformerNMT, _nmt_batch, _nmt_loss, 512, "rmsprop", dict(lr=1e-3),
                            samples_unit="tok", tokens_per_sample=20),
    "bert-base": Workload("bert-base", BertBase, _bert_batch, _bert_loss, 32, "adamw",
                          dict(lr=1e-4, weight_decay=0.01), samples_unit="tok", tokens_per_sample=128),
}


def get_workload(name: str) -> Workload:
    try:
        return WORKLOADS[name]
    except KeyError:
        raise KeyError(f"unknown workload {name!r}; known: {sorted(WORKLOADS)}") from None


__all__ = ["WORKLOADS", "Workload", "get_workload", "resnet50", "resnet18", "vgg16_cifar", "InceptionV3",
           "KerasMnistCNN", "TorchMnistNet", "TransformerNMT", "BertBase"]
