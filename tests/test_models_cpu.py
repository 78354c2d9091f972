"""Model zoo parity with the reference workloads (SURVEY.md §2.8 parameter counts, counted the
Keras way: weights + BatchNorm moving statistics)."""
import pytest
import torch

from vodascheduler_amd.models import WORKLOADS
from vodascheduler_amd.models.convnets import keras_param_count


@pytest.mark.parametrize("name,count", [
    ("inceptionv3", 21_823_274),   # applications.InceptionV3(classes=10): 23,851,784 - 2,049,000 + 20,490
    ("vgg16", 33_638_218),         # applications.VGG16(classes=10) at 32x32
    ("mnist", 1_199_882),          # tensorflow2_keras_mnist_elastic.py:101-110
    ("mnist-torch", 21_840),       # pytorch_mnist_elastic.py:80-96
    ("transformer", 19_960_216),   # neural_machine_translation_with_transformer.py
])
def test_reference_parameter_counts(name, count):
    assert keras_param_count(WORKLOADS[name].build()) == count


def test_inceptionv3_full_topology_shapes():
    m = WORKLOADS["inceptionv3"].build().eval()
    feats = {}
    m.a.register_forward_hook(lambda mod, i, o: feats.__setitem__("a", o.shape))
    m.c.register_forward_hook(lambda mod, i, o: feats.__setitem__("c", o.shape))
    m.d.register_forward_hook(lambda mod, i, o: feats.__setitem__("d", o.shape))
    m.e.register_forward_hook(lambda mod, i, o: feats.__setitem__("e", o.shape))
    with torch.no_grad():
        y = m(torch.randn(2, 3, 75, 75))
    assert y.shape == (2, 10)
    assert feats == {"a": (2, 288, 7, 7), "c": (2, 768, 3, 3), "d": (2, 1280, 1, 1), "e": (2, 2048, 1, 1)}
    # Keras conv2d_bn: BatchNormalization(scale=False) -> no gamma
    assert m.stem[0].bn.weight is None and m.stem[0].bn.bias is not None
