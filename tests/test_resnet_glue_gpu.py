"""ResNet glue kernels (csrc/hip/pool.hip): stride-s pixel subsampling of channels_last bf16 /
fp32 tensors (the stride-2 1x1 downsample input) and its adjoint, against PyTorch slicing."""
import pytest
import torch

from vodascheduler_amd.ops.conv1x1 import subsample, subsample_add_

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape,s", [((4, 256, 56, 56), 2), ((3, 64, 17, 13), 2), ((2, 8, 9, 10), 3), ((1, 16, 1, 1), 2)])
def test_subsample_gather_and_add_exact(shape, s, dtype):
    torch.manual_seed(0)
    cl = torch.channels_last
    x = torch.randn(shape, device="cuda").to(dtype).to(memory_format=cl)
    y = subsample(x, s)
    assert y.is_contiguous(memory_format=cl)
    assert torch.equal(y, x[:, :, ::s, ::s])
    g = torch.randn_like(y)
    dx = x.clone()
    subsample_add_(dx, g, s)
    want = x.clone()
    want[:, :, ::s, ::s] += g
    assert torch.equal(dx, want)


def test_subsample_falls_back_for_other_layouts():
    x = torch.randn(2, 12, 8, 8, device="cuda").bfloat16()  # NCHW, C % 8 != 0
    assert torch.equal(subsample(x, 2), x[:, :, ::2, ::2])
