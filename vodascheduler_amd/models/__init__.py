"""Model zoo + synthetic-data workload registry.

Every workload of the reference (W1 ResNet50/VGG16/InceptionV3 on CIFAR-10,
W2 Keras MNIST CNN, W3 Transformer NMT, W4 PyTorch MNIST) plus the BASELINE configs'
ResNet-50 ImageNet-shape and BERT-base, with random-init weights and synthetic batches of the
real shapes (no datasets are available offline).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Callable

import torch
import torch.nn.functional as F

from ..ops.xent import softmax_cross_entropy
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
    # whole-step hipGraph capture validated on MI355X (benchmarks/graph_diag.py: replayed
    # gradients == eager, real-update trajectories match; tests/test_stepgraph_gpu.py).  Not
    # for models with library paths that are not capture-safe (InceptionV3's MIOpen backward
    # solvers; docs/kernels.md)
    graph_safe: bool = False
    # (loss, #correct predictions, #predictions) of one batch, all device tensors: the
    # training step logs accuracy from the same forward (Keras ``metrics=["accuracy"]``,
    # reference tensorflow2_keras_cifar_elastic.py:168) and the eval pass (reference
    # pytorch_mnist_elastic.py:155-176 ``test()``) sums them across ranks
    metrics: Callable[[torch.nn.Module, tuple], tuple] | None = None

    def loss_metrics(self, model: torch.nn.Module, batch: tuple) -> tuple:
        if self.metrics is not None:
            return self.metrics(model, batch)
        loss = self.loss(model, batch)
        z = torch.zeros((), device=loss.device)
        return loss, z, z


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


def _cls_metrics(log_probs: bool = False):
    def f(model, batch):
        x, y = batch
        out = model(x).float()
        loss = F.nll_loss(out, y) if log_probs else F.cross_entropy(out, y)
        correct = (out.argmax(1) == y).sum()
        return loss, correct, torch.full((), y.numel(), device=y.device)
    return f


def _nmt_metrics(model, batch):
    """Loss over real tokens (padding id 0 ignored) and the reference's masked accuracy, from
    one fused cross-entropy pass over the vocab logits (ops/xent.py)."""
    src, tin, tout = batch
    logits = model(src, tin)
    return softmax_cross_entropy(logits.reshape(-1, logits.shape[-1]), tout.reshape(-1),
                                 getattr(model, "num_classes", None), ignore_index=0)


def _bert_metrics(model, batch):
    ids, mask, pos, labels = batch
    logits = model(ids, mask, pos)
    return softmax_cross_entropy(logits, labels.reshape(-1), getattr(model, "num_classes", None))


def _nmt_batch(b, dev, g=None, vocab=15000, T=20):
    src = torch.randint(1, vocab, (b, T), device=dev, generator=g)
    tgt = torch.randint(1, vocab, (b, T + 1), device=dev, generator=g)
    src[:, -3:] = 0  # some padding, as in the reference's padded sentences
    return src, tgt[:, :-1], tgt[:, 1:]


def _nmt_loss(model, batch):
    return _nmt_metrics(model, batch)[0]


def _bert_batch(b, dev, g=None, vocab=30522, T=128, P=20):
    """BERT pretraining batch in the reference input format: input ids, attention mask,
    ``masked_lm_positions`` [B, P] and ``masked_lm_ids`` [B, P] (P = max_predictions_per_seq
    = 20 for seq 128, i.e. 15 % masking)."""
    ids = torch.randint(1000, vocab, (b, T), device=dev, generator=g)
    mask = torch.ones(b, T, device=dev, dtype=torch.bool)
    pos = torch.argsort(torch.rand(b, T - 1, device=dev, generator=g), dim=1)[:, :P] + 1  # never [CLS]
    pos = torch.sort(pos, dim=1).values
    labels = torch.gather(ids, 1, pos)
    return ids, mask, pos, labels


def _bert_loss(model, batch):
    return _bert_metrics(model, batch)[0]


_CE, _NLL = _cls_metrics(), _cls_metrics(log_probs=True)

WORKLOADS: dict[str, Workload] = {
    "resnet50": Workload("resnet50", lambda: resnet50(1000), _img_batch(3, 224, 224, 1000), _ce, 256, "sgd",
                         dict(lr=0.1, momentum=0.9, weight_decay=5e-5), channels_last=True, metrics=_CE),
    "resnet50-cifar": Workload("resnet50-cifar", lambda: resnet50(10, small_input=True), _img_batch(3, 32, 32, 10),
                               _ce, 128, "sgd", dict(lr=0.01, momentum=0.9), channels_last=True, metrics=_CE,
                               graph_safe=True),  # 14.33 -> 7.86 ms per step as a graph
    "resnet18": Workload("resnet18", lambda: resnet18(1000), _img_batch(3, 224, 224, 1000), _ce, 256, "sgd",
                         dict(lr=0.1, momentum=0.9), channels_last=True, metrics=_CE),
    "vgg16": Workload("vgg16", vgg16_cifar, _img_batch(3, 32, 32, 10), _ce, 128, "sgd",
                      dict(lr=0.01, momentum=0.9), channels_last=True, metrics=_CE,
                      graph_safe=True),  # conv bias on ops/conv_bias.py: 2.63 -> 2.36 ms as a graph
    "inceptionv3": Workload("inceptionv3", InceptionV3, _img_batch(3, 75, 75, 10), _ce, 128, "rmsprop",
                            dict(lr=1e-3), channels_last=True, metrics=_CE),
    "mnist": Workload("mnist", KerasMnistCNN, _img_batch(1, 28, 28, 10), _ce, 128, "adam", dict(lr=1e-3),
                      graph_safe=True, metrics=_CE),
    "mnist-torch": Workload("mnist-torch", TorchMnistNet, _img_batch(1, 28, 28, 10), _nll, 64, "sgd",
                            dict(lr=0.01, momentum=0.5), graph_safe=True, metrics=_NLL),
    "transformer": Workload("transformer", TransformerNMT, _nmt_batch, _nmt_loss, 512, "rmsprop", dict(lr=1e-3),
                            samples_unit="tok", tokens_per_sample=20, metrics=_nmt_metrics),
    "bert-base": Workload("bert-base", BertBase, _bert_batch, _bert_loss, 64, "adamw",
                          dict(lr=1e-4, weight_decay=0.01), samples_unit="tok", tokens_per_sample=128,
                          metrics=_bert_metrics,
                          # replays exact at bs 64 once the embeddings' backward is the flat-gradient
                          # column-sum / index_add path (check 31: frozen grads bitwise, 5-step
                          # trajectory equal); 11.0-11.28 -> 10.75 ms per step as a graph
                          graph_safe=True),
}


def cast_compute_weights_(model: torch.nn.Module, dtype: torch.dtype = torch.bfloat16) -> torch.nn.Module:
    """Store GEMM / convolution / embedding weights (and Linear biases) in ``dtype``.

    Under bf16 autocast those weights are otherwise re-cast from fp32 on every forward and
    their gradients cast back and accumulated in fp32 -- ~3 small kernels per parameter per
    step (measured: ~4 ms of a 25 ms BERT-base step, profiles/).  Normalisation parameters
    stay fp32.  The fused optimizers keep an fp32 master copy of every bf16 parameter and
    write the bf16 model copy in the same pass, so the update precision is unchanged.
    Parameter identity is kept (tied weights stay tied)."""
    seen: set[int] = set()
    for m in model.modules():
        if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d, torch.nn.Conv1d, torch.nn.Embedding)):
            for p in m.parameters(recurse=False):
                if id(p) not in seen and p.dtype.is_floating_point:
                    seen.add(id(p))
                    p.data = p.data.to(dtype)
    return model


def prepare_model(w: "Workload", device: torch.device, amp: bool = True) -> torch.nn.Module:
    """Build a workload's model on ``device`` in the layout/precision the trainer uses:
    channels_last for convnets, bf16 compute weights on GPU with autocast."""
    m = w.build().to(device)
    if w.channels_last and device.type == "cuda":
        m = m.to(memory_format=torch.channels_last)
        # MIOpen exhaustive find once per conv shape (cached in-process and in MIOpen's
        # find-db, so warm pool workers pay it once): ResNet-50 bs256 step 34.6 -> 31.0 ms
        torch.backends.cudnn.benchmark = True
    if amp and device.type == "cuda":
        cast_compute_weights_(m, torch.bfloat16)
        from ..utils.tunable import configure as _tunable

        _tunable("bf16")  # pre-tuned hipBLASLt solutions of the bf16 GEMMs, when shipped
    elif device.type == "cuda":
        # reference precision: true fp32 math in the library GEMMs / convolutions too
        torch.backends.cuda.matmul.allow_tf32 = False
        torch.backends.cudnn.allow_tf32 = False
        # pre-tuned hipBLASLt solutions of the fp32 GEMMs (utils/tunable.py)
        from ..utils.tunable import configure as _tunable

        _tunable("fp32")
    return m


def get_workload(name: str) -> Workload:
    try:
        return WORKLOADS[name]
    except KeyError:
        raise KeyError(f"unknown workload {name!r}; known: {sorted(WORKLOADS)}") from None


__all__ = ["WORKLOADS", "Workload", "get_workload", "prepare_model", "cast_compute_weights_", "resnet50", "resnet18", "vgg16_cifar", "InceptionV3",
           "KerasMnistCNN", "TorchMnistNet", "TransformerNMT", "BertBase"]
