"""Implicit-GEMM convolution weight gradient (csrc/hip/wgrad.hip ``wgrad_conv``,
ops/conv3x3.py) against the fp32 PyTorch reference (torch.nn.grad.conv2d_weight): ResNet
3x3 shapes, stride 2, odd image sizes and channel counts off the 128 tile, every split count,
overwrite and accumulate; plus the ConvKxK layer through a flat-gradient optimizer."""
import pytest
import torch
import torch.nn.functional as F

from vodascheduler_amd.ops import conv3x3 as C


def test_cpu_reference_path_and_fallback_layer():
    torch.manual_seed(0)
    x = torch.randn(2, 8, 9, 11)
    dy = torch.randn(2, 16, 5, 6)
    gw = torch.randn(16, 8, 3, 3)
    want = torch.nn.grad.conv2d_weight(x, gw.shape, dy, stride=2, padding=1) + gw
    C.conv_wgrad_accumulate_(dy, x, gw, 2, 1)
    torch.testing.assert_close(gw, want, rtol=1e-4, atol=1e-4)
    m = C.ConvKxK(8, 16, 3, stride=2, padding=1)
    torch.testing.assert_close(m(x), F.conv2d(x, m.weight, stride=2, padding=1))
    assert set(m.state_dict()) == {"weight"}


def _case(n, cin, cout, h, w, stride, pad=1, k=3, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    cl = torch.channels_last
    x = (torch.randn(n, cin, h, w, device="cuda", generator=g)
         + torch.arange(cin, device="cuda").view(1, cin, 1, 1) / cin).bfloat16().to(memory_format=cl)
    ho = (h + 2 * pad - k) // stride + 1
    wo = (w + 2 * pad - k) // stride + 1
    dy = torch.randn(n, cout, ho, wo, device="cuda", generator=g).bfloat16().to(memory_format=cl)
    gw = torch.randn(cout, cin, k, k, device="cuda", generator=g).bfloat16().to(memory_format=cl)
    return dy, x, gw


@pytest.mark.gpu
@pytest.mark.parametrize("n,cin,cout,h,w,stride", [(2, 64, 64, 56, 56, 1), (2, 128, 128, 56, 56, 2),
                                                   (4, 256, 256, 14, 14, 1), (8, 512, 512, 7, 7, 1),
                                                   (3, 24, 40, 9, 11, 2), (2, 136, 72, 13, 5, 1)])
@pytest.mark.parametrize("splits", [1, 3, 16])
def test_conv_wgrad_matches_fp32(n, cin, cout, h, w, stride, splits):
    dy, x, gw = _case(n, cin, cout, h, w, stride)
    want = C.conv_wgrad_ref(dy, x, gw.shape, stride, 1) + gw.float()
    got = gw.clone()
    C.conv_wgrad_accumulate_(dy, x, got, stride, 1, splits=splits)
    torch.cuda.synchronize()
    rel = float((got.float() - want).norm() / want.norm())
    assert rel < 1e-2, rel
    # overwrite mode
    got2 = gw.clone()
    C.conv_wgrad_accumulate_(dy, x, got2, stride, 1, accumulate=False, splits=splits)
    want2 = C.conv_wgrad_ref(dy, x, gw.shape, stride, 1)
    assert float((got2.float() - want2).norm() / want2.norm()) < 1e-2


@pytest.mark.gpu
def test_conv_wgrad_single_tap_exact():
    # dY = one-hot at output pixel (0, 3, 4), X arbitrary: dW[:, :, kh, kw] = X at the tapped
    # input pixel (bf16 values, fp32 sums of one term: exact), zero where the tap falls outside
    dy, x, gw = _case(1, 16, 8, 6, 7, 1, seed=2)
    dy.zero_()
    dy[0, :, 3, 4] = 1
    got = torch.zeros_like(gw)
    C.conv_wgrad_accumulate_(dy, x, got, 1, 1, accumulate=False, splits=1)
    want = C.conv_wgrad_ref(dy, x, gw.shape, 1, 1).to(torch.bfloat16)
    torch.testing.assert_close(got, want, rtol=0, atol=0)


@pytest.mark.gpu
def test_convkxk_layer_flat_grads_match_autograd():
    from vodascheduler_amd.ops.optim import make_optimizer

    torch.manual_seed(0)
    cl = torch.channels_last
    m = C.ConvKxK(128, 128, 3, stride=2, padding=1).cuda().to(memory_format=cl).bfloat16()
    ref_w = m.weight.detach().float().clone().requires_grad_(True)
    opt = make_optimizer("sgd", m.parameters(), lr=0.0)  # flat fp32 grads: kernel path
    x = torch.randn(8, 128, 28, 28, device="cuda").bfloat16().to(memory_format=cl)
    xg = x.detach().requires_grad_(True)
    xr = x.float().detach().requires_grad_(True)
    assert m._fast_ok(xg)
    opt.zero_grad()
    y = m(xg)
    yr = F.conv2d(xr, ref_w, stride=2, padding=1)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16().to(memory_format=cl))
    yr.backward(g)
    from vodascheduler_amd.utils.flat import grad_of

    for got, want in ((grad_of(m.weight), ref_w.grad), (xg.grad, xr.grad)):
        rel = float((got.float() - want).norm() / want.norm())
        assert rel < 1e-2, rel


@pytest.mark.gpu
@pytest.mark.parametrize("n,cin,cout,h,w,stride", [(2, 128, 128, 56, 56, 2), (4, 256, 256, 14, 14, 1)])
@pytest.mark.parametrize("splits", [1, 16])
def test_conv_wgrad_fp32_output(n, cin, cout, h, w, stride, splits):
    """fp32 weight gradient (the default flat-gradient precision of a bf16 model)."""
    dy, x, gw = _case(n, cin, cout, h, w, stride, seed=2)
    g32 = gw.float().contiguous(memory_format=torch.channels_last)
    want = C.conv_wgrad_ref(dy, x, gw.shape, stride, 1) + g32
    C.conv_wgrad_accumulate_(dy, x, g32, stride, 1, splits=splits)
    torch.cuda.synchronize()
    rel = float((g32 - want).norm() / want.norm())
    assert rel < 1e-4, rel
