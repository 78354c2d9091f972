"""ResNet stem (ops/stem.py, csrc/hip/stem.hip): the NHWC-4 pack, the MFMA 7x7/2 conv with
BN statistics in its epilogue, and the whole conv + BN + ReLU + max-pool training op
against the PyTorch fp32 composition."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from vodascheduler_amd.ops import stem as S
from vodascheduler_amd.ops.batchnorm import FusedBNReLUMaxPool2d


def test_fused_stem_cpu_is_the_composition():
    torch.manual_seed(0)
    m = S.FusedStem(3, 64)
    ref = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), FusedBNReLUMaxPool2d(64, 3, 2, 1))
    assert set(m.state_dict()) == set(ref.state_dict())
    ref.load_state_dict(m.state_dict())
    x = torch.randn(2, 3, 40, 36)
    torch.testing.assert_close(m(x), ref(x))
    m.eval(), ref.eval()
    torch.testing.assert_close(m(x), ref(x))


def _img(n, h, w, dtype=torch.float32, cl=False, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(n, 3, h, w, device="cuda", generator=g).to(dtype)
    return x.to(memory_format=torch.channels_last) if cl else x


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,cl,w", [(torch.float32, False, 21), (torch.float32, False, 224),
                                        (torch.float32, True, 24), (torch.float32, True, 22),
                                        (torch.bfloat16, True, 21),
                                        (torch.float16, False, 21)])
def test_pack_nhwc4_exact(dtype, cl, w):
    """Generic and 4-pixel-vectorised (fp32 NCHW, W % 4 == 0) pack kernels."""
    x = _img(3, 17, w, dtype, cl)
    x4 = S.pack_nhwc4(x)
    want = F.pad(x.float().permute(0, 2, 3, 1), (0, 1)).bfloat16()
    assert torch.equal(x4, want)


def _conv_ref(x, w):
    """fp32 conv of the bf16-rounded operands (what the MFMA kernel multiplies)."""
    return F.conv2d(x.bfloat16().float(), w.float(), stride=2, padding=3)


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w", [(2, 224, 224), (8, 224, 224), (3, 97, 61), (1, 256, 255), (2, 9, 1)])
def test_stem_conv_and_partial_stats_vs_fp32(n, h, w):
    torch.manual_seed(1)
    x = _img(n, h, w)
    wt = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).bfloat16()
    x4 = S.pack_nhwc4(x)
    y, ws, nb = S.stem_conv_stats(x4, wt, 3)
    ref = _conv_ref(x, wt)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), ref, rtol=8e-3, atol=8e-3 * ref.abs().max().item())
    part = ws[: 2 * nb * 64].view(2, nb, 64).double().sum(1)
    yd = ref.double()
    torch.testing.assert_close(part[0], yd.sum((0, 2, 3)), rtol=1e-4, atol=1e-3 * yd.numel() ** 0.5)
    torch.testing.assert_close(part[1], (yd * yd).sum((0, 2, 3)), rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
def test_stem_conv_weight_layouts():
    """Any filter strides (the kernel gathers its fragments once per workgroup)."""
    torch.manual_seed(2)
    x = _img(2, 64, 64)
    w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).bfloat16()
    x4 = S.pack_nhwc4(x)
    y0, _, _ = S.stem_conv_stats(x4, w, 3)
    y1, _, _ = S.stem_conv_stats(x4, w.contiguous(memory_format=torch.channels_last), 3)
    assert torch.equal(y0, y1)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,cl", [(torch.float32, False), (torch.bfloat16, True)])
def test_fused_stem_training_step_vs_composition(dtype, cl):
    """Forward output, running statistics and the gradients of the conv filter and the BN
    affine parameters: FusedStem (HIP) vs the composition on the same bf16 filter."""
    torch.manual_seed(3)
    m = S.FusedStem(3, 64).cuda()
    ref = S.FusedStem(3, 64).cuda()
    ref.load_state_dict(m.state_dict())
    for mod in (m, ref):
        mod[0].weight.data = mod[0].weight.data.bfloat16().contiguous(memory_format=torch.channels_last)
        mod[1].weight.data.uniform_(0.5, 1.5)
    ref[1].weight.data.copy_(m[1].weight.data)
    x = _img(4, 224, 224, dtype, cl, seed=4)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert m._fast_ok(x)
        y = m(x)
        assert type(y.grad_fn).__name__ == "_StemFnBackward"
    # reference: the same ops, fp32 conv of the bf16-rounded operands, fused BN/pool
    xr = x.bfloat16().float()
    yc = F.conv2d(xr, ref[0].weight.float(), stride=2, padding=3).bfloat16().contiguous(
        memory_format=torch.channels_last)
    yr = ref[1](yc)
    torch.testing.assert_close(y.float(), yr.float(), rtol=3e-2, atol=3e-2)
    m[1].sync_batches_tracked()
    torch.testing.assert_close(m[1].running_mean, ref[1].running_mean, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(m[1].running_var, ref[1].running_var, rtol=1e-3, atol=1e-4)
    assert int(m[1].num_batches_tracked) == 1
    dy = torch.randn_like(y)
    y.backward(dy)
    w32 = ref[0].weight.detach().float().requires_grad_()
    yc2 = F.conv2d(xr, w32, stride=2, padding=3)
    ref[1].zero_grad()
    yr2 = ref[1](yc2.bfloat16().contiguous(memory_format=torch.channels_last))
    yr2.backward(dy.to(yr2.dtype))
    gw = m[0].weight.grad.float()
    torch.testing.assert_close(gw, w32.grad, rtol=3e-2, atol=3e-2 * w32.grad.abs().max().item())
    torch.testing.assert_close(m[1].weight.grad, ref[1].weight.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(m[1].bias.grad, ref[1].bias.grad, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_resnet50_uses_fused_stem():
    from vodascheduler_amd.models.resnet import resnet50

    m = resnet50().cuda().to(memory_format=torch.channels_last)
    assert isinstance(m.stem, S.FusedStem)
    x = _img(2, 224, 224)
    m.stem[0].weight.data = m.stem[0].weight.data.bfloat16()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert m.stem._fast_ok(x)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_global_avgpool_backward_channels_last(dt):
    from vodascheduler_amd.ops.pool import GlobalAvgPool2d

    torch.manual_seed(5)
    x = torch.randn(4, 64, 7, 7, device="cuda").to(dt).to(memory_format=torch.channels_last).requires_grad_()
    y = GlobalAvgPool2d()(x)
    assert type(y.grad_fn).__name__ == "_GlobalAvgPoolFnBackward"
    torch.testing.assert_close(y.float(), x.float().mean((2, 3), keepdim=True), rtol=1e-2, atol=1e-2)
    g = torch.randn(4, 64, 1, 1, device="cuda").to(dt)
    y.backward(g)
    want = (g.float() / 49).expand(4, 64, 7, 7)
    assert x.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(x.grad.float(), want, rtol=1e-2, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w", [(2, 224, 224), (3, 97, 61), (1, 256, 255), (5, 30, 30)])
@pytest.mark.parametrize("out", ["fp32_acc", "bf16"])
def test_stem_wgrad_vs_fp64(n, h, w, out):
    """dW of the 7x7/2 conv from the packed image and a bf16 dY (MFMA kernel, fp32 partials,
    two-pass reduce) against the fp64 conv2d_weight of the same bf16 operands."""
    torch.manual_seed(6)
    x = _img(n, h, w)
    x4 = S.pack_nhwc4(x)
    ho, wo = S._out(h), S._out(w)
    dy = torch.randn(n, 64, ho, wo, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    want = torch.nn.grad.conv2d_weight(x.bfloat16().double(), (64, 3, 7, 7), dy.double(), stride=2, padding=3)
    hip = S.N.hip()
    ws = torch.empty(hip.stem_wgrad_workspace_floats(n, ho), dtype=torch.float32, device="cuda")
    if out == "fp32_acc":
        base = torch.randn(64, 3, 7, 7, device="cuda").contiguous(memory_format=torch.channels_last)
        dw = base.clone()
        hip.stem_conv_wgrad(x4.data_ptr(), dy.data_ptr(), dw.data_ptr(), *dw.stride(), 3, ws.data_ptr(), n, h, w,
                            ho, wo, True, S.N.dtype_code(dw.dtype), S.N.stream_of(x4))
        got = (dw - base).double()
        tol = 1e-4 * want.abs().max().item()
    else:
        dw = torch.empty(64, 3, 7, 7, device="cuda", dtype=torch.bfloat16)
        hip.stem_conv_wgrad(x4.data_ptr(), dy.data_ptr(), dw.data_ptr(), *dw.stride(), 3, ws.data_ptr(), n, h, w,
                            ho, wo, False, S.N.dtype_code(dw.dtype), S.N.stream_of(x4))
        got = dw.double()
        tol = 1e-2 * want.abs().max().item()
    torch.testing.assert_close(got, want, rtol=1e-2, atol=tol)


# ---------------------------------------------------------------- fp32 stem (stem_f32.hip)
@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w,cl", [(2, 224, 224, False), (2, 224, 224, True), (3, 97, 61, False),
                                      (1, 256, 255, True), (2, 9, 1, False), (5, 40, 36, False)])
def test_stem_conv_f32_and_partial_stats_vs_fp64(n, h, w, cl):
    """fp32 MFMA 7x7/2 convolution read straight from the image's strides (NCHW or
    channels_last), ragged output widths, with the BN partial sums of its epilogue."""
    torch.manual_seed(1)
    x = _img(n, h, w, cl=cl)
    wt = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    y, ws, nb = S.stem_conv_stats_f32(x, wt)
    ref = F.conv2d(x.double(), wt.double(), stride=2, padding=3)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-5 * ref.abs().max().item())
    part = ws[: 2 * nb * 64].view(2, nb, 64).double().sum(1)
    torch.testing.assert_close(part[0], ref.sum((0, 2, 3)), rtol=1e-5, atol=1e-4 * ref.numel() ** 0.5)
    torch.testing.assert_close(part[1], (ref * ref).sum((0, 2, 3)), rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
def test_stem_conv_f32_weight_layouts_and_channels():
    """Any filter strides; fewer than 3 input channels (the missing ones read as zero)."""
    torch.manual_seed(2)
    x = _img(2, 64, 64)
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    y0, _, _ = S.stem_conv_stats_f32(x, w)
    y1, _, _ = S.stem_conv_stats_f32(x, w.contiguous(memory_format=torch.channels_last))
    assert torch.equal(y0, y1)
    x1 = x[:, :1].contiguous()
    y2, _, _ = S.stem_conv_stats_f32(x1, w[:, :1].contiguous())
    ref = F.conv2d(x1.double(), w[:, :1].double(), stride=2, padding=3)
    torch.testing.assert_close(y2.double(), ref, rtol=1e-5, atol=1e-5 * ref.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("cl", [False, True])
def test_fused_stem_fp32_training_step_vs_composition(cl):
    """fp32 FusedStem (own conv + statistics epilogue, fused BN/pool, MIOpen weight gradient)
    vs the plain fp32 composition: output, running statistics, filter and BN gradients."""
    torch.manual_seed(3)
    m = S.FusedStem(3, 64).cuda()
    ref = S.FusedStem(3, 64).cuda()
    m[1].weight.data.uniform_(0.5, 1.5)
    ref.load_state_dict(m.state_dict())
    x = _img(4, 224, 224, cl=cl, seed=4)
    assert m._fast_f32_ok(x)
    y = m(x)
    assert type(y.grad_fn).__name__ == "_StemF32FnBackward"
    yc = F.conv2d(x, ref[0].weight, stride=2, padding=3).contiguous(memory_format=torch.channels_last)
    yr = ref[1](yc)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    m[1].sync_batches_tracked()
    ref[1].sync_batches_tracked()
    torch.testing.assert_close(m[1].running_mean, ref[1].running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m[1].running_var, ref[1].running_var, rtol=1e-5, atol=1e-6)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy)
    for a, b in ((m[0].weight.grad, ref[0].weight.grad), (m[1].weight.grad, ref[1].weight.grad),
                 (m[1].bias.grad, ref[1].bias.grad)):
        rel = ((a - b).norm() / b.norm()).item()
        assert rel < 1e-4, rel


@pytest.mark.gpu
def test_resnet50_fp32_uses_fused_stem_f32():
    from vodascheduler_amd.models.resnet import resnet50

    m = resnet50().cuda().to(memory_format=torch.channels_last)
    x = _img(2, 224, 224, cl=True)
    assert m.stem._fast_f32_ok(x) and not m.stem._fast_ok(x)


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w,cl,acc", [(2, 224, 224, True, False), (3, 97, 61, False, True),
                                          (1, 30, 223, True, False), (4, 9, 1, False, False)])
def test_stem_wgrad_f32_vs_fp64(n, h, w, cl, acc):
    """Own fp32 filter gradient (pixel reduction on the f32 MFMA) against fp64, any image
    strides, odd / ragged output widths, (+)= into an existing gradient."""
    torch.manual_seed(5)
    x = _img(n, h, w, cl=cl, seed=5)
    ho, wo = S._out(h), S._out(w)
    dy = torch.randn(n, 64, ho, wo, device="cuda").contiguous(memory_format=torch.channels_last)
    wt = torch.randn(64, 3, 7, 7, device="cuda")
    from vodascheduler_amd.ops import _native as N

    hh = N.hip()
    ws = torch.empty(hh.stem_wgrad_f32_workspace_floats(n, ho), device="cuda")
    base = torch.randn_like(wt) if acc else torch.zeros_like(wt)
    out = base.clone()
    hh.stem_conv_wgrad_f32(x.data_ptr(), *x.stride(), 3, dy.data_ptr(), out.data_ptr(), *out.stride(),
                           ws.data_ptr(), n, h, w, ho, wo, acc, N.stream_of(x))
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_weight(x.double(), wt.shape, dy.double(), stride=2, padding=3)
    if acc:
        ref = ref + base.double()
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-5 * ref.abs().max().item())
