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


@pytest.mark.parametrize("k,pad", [(3, 1), (3, 0), (5, 2), (7, 3), (1, 0)])
def test_dgrad_as_forward_matches_conv2d_input(k, pad):
    """dX of a stride-1 convolution == forward convolution of dY with the flipped,
    channel-transposed filter (the VODA_CONV_DGRAD_FWD path), fp64 on the CPU."""
    torch.manual_seed(k)
    x = torch.randn(2, 6, 9, 11, dtype=torch.float64)
    w = torch.randn(10, 6, k, k, dtype=torch.float64)
    dy = torch.randn_like(F.conv2d(x, w, padding=pad))
    want = torch.nn.grad.conv2d_input(x.shape, w, dy, stride=1, padding=pad)
    torch.testing.assert_close(C.dgrad_as_forward(dy, w, pad), want)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [3, 1, 5])
@pytest.mark.parametrize("wdt,odt", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                     (torch.bfloat16, torch.bfloat16)])
@pytest.mark.parametrize("cl", [True, False])
def test_flipped_filter_kernel_matches_torch(k, wdt, odt, cl):
    """One-launch flipped, channel-transposed filter (filter_flip_t) == the torch composition,
    bitwise, for channels_last and contiguous weights."""
    torch.manual_seed(k)
    w = torch.randn(48, 40, k, k, device="cuda").to(wdt)
    if cl:
        w = w.contiguous(memory_format=torch.channels_last)
    got = C.flipped_filter(w, odt)
    want = w.transpose(0, 1).flip(2, 3).to(odt)
    assert got.shape == want.shape and got.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout", [(64, 64), (128, 128)])
def test_convkxk_dgrad_forward_path_matches_autograd(monkeypatch, cin, cout):
    """The ConvKxK layer with VODA_CONV_DGRAD_FWD on: bf16 input gradient == stock autograd's
    (both are MIOpen bf16 convolutions; tolerance of bf16 rounding of the result)."""
    monkeypatch.setattr(C, "DGRAD_FWD", True)
    torch.manual_seed(0)
    cl = torch.channels_last
    m = C.ConvKxK(cin, cout, 3, stride=1, padding=1).cuda().bfloat16().to(memory_format=cl)
    x = torch.randn(4, cin, 28, 28, device="cuda").bfloat16().to(memory_format=cl).requires_grad_()
    y = m(x)
    assert type(y.grad_fn).__name__.startswith("_ConvKxKFn")
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    F.conv2d(xr, m.weight.float(), padding=1).backward(dy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=2e-2 * xr.grad.abs().max().item())
    assert m.weight.grad is not None


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w", [(2, 56, 56), (3, 17, 9), (1, 5, 64), (4, 30, 64), (2, 1, 1)])
@pytest.mark.parametrize("out", ["fp32_acc", "bf16"])
def test_conv3x3_c64_wgrad_vs_fp64(n, h, w, out):
    """64 -> 64 3x3 / stride-1 weight gradient (csrc/hip/conv3x3_c64.hip): transposed-LDS-read
    MFMA GEMM over the pixels, fp32 partials, two-pass reduce, vs fp64 conv2d_weight."""
    torch.manual_seed(7)
    cl = torch.channels_last
    x = torch.randn(n, 64, h, w, device="cuda").bfloat16().to(memory_format=cl)
    dy = torch.randn(n, 64, h, w, device="cuda").bfloat16().to(memory_format=cl)
    want = torch.nn.grad.conv2d_weight(x.double(), (64, 64, 3, 3), dy.double(), stride=1, padding=1)
    hip = C.N.hip()
    ws = torch.empty(hip.conv3x3_c64_wgrad_workspace_floats(n, h), dtype=torch.float32, device="cuda")
    if out == "fp32_acc":
        base = torch.randn(64, 64, 3, 3, device="cuda").contiguous(memory_format=cl)
        dw = base.clone()
        hip.conv3x3_c64_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), *dw.stride(), ws.data_ptr(), n, h, w,
                              True, C.N.dtype_code(dw.dtype), C.N.stream_of(x), C.N.dtype_code(x.dtype))
        got, tol = (dw - base).double(), 1e-4
    else:
        dw = torch.empty(64, 64, 3, 3, device="cuda", dtype=torch.bfloat16)
        hip.conv3x3_c64_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), *dw.stride(), ws.data_ptr(), n, h, w,
                              False, C.N.dtype_code(dw.dtype), C.N.stream_of(x), C.N.dtype_code(x.dtype))
        got, tol = dw.double(), 1e-2
    torch.testing.assert_close(got, want, rtol=1e-2, atol=tol * want.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w", [(2, 56, 56), (3, 17, 9), (1, 5, 64), (4, 30, 63), (2, 1, 1), (16, 56, 56)])
def test_conv3x3_c64_wgrad_f32_vs_fp64(n, h, w):
    """fp32 twin of the 64-channel 3x3 weight gradient (f32 MFMA: exact products, fp32 sums):
    fp32 accumulation into a base and plain output vs fp64 conv2d_weight."""
    torch.manual_seed(9)
    cl = torch.channels_last
    x = torch.randn(n, 64, h, w, device="cuda").to(memory_format=cl)
    dy = torch.randn(n, 64, h, w, device="cuda").to(memory_format=cl)
    want = torch.nn.grad.conv2d_weight(x.double(), (64, 64, 3, 3), dy.double(), stride=1, padding=1)
    hip = C.N.hip()
    ws = torch.empty(hip.conv3x3_c64_wgrad_workspace_floats(n, h), dtype=torch.float32, device="cuda")
    base = torch.randn(64, 64, 3, 3, device="cuda").contiguous(memory_format=cl)
    dw = base.clone()
    hip.conv3x3_c64_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), *dw.stride(), ws.data_ptr(), n, h, w, True,
                          C.N.dtype_code(dw.dtype), C.N.stream_of(x), C.N.dtype_code(x.dtype))
    rel = float(((dw - base).double() - want).norm() / want.norm())
    assert rel < 1e-5, rel
    out = torch.full((64, 64, 3, 3), float("nan"), device="cuda")
    hip.conv3x3_c64_wgrad(x.data_ptr(), dy.data_ptr(), out.data_ptr(), *out.stride(), ws.data_ptr(), n, h, w, False,
                          C.N.dtype_code(out.dtype), C.N.stream_of(x), C.N.dtype_code(x.dtype))
    assert float((out.double() - want).norm() / want.norm()) < 1e-5


@pytest.mark.gpu
def test_convkxk_c64_fp32_layer_uses_kernel(monkeypatch):
    """fp32 64-channel ConvKxK under a flat-gradient optimizer: weight gradient from the fp32
    c64 kernel into the flat buffer (tight vs fp64), input gradient as a forward conv."""
    from vodascheduler_amd.ops.optim import make_optimizer
    from vodascheduler_amd.utils.flat import grad_of

    monkeypatch.setattr(C, "USE_C64_WGRAD_F32", True)
    torch.manual_seed(10)
    cl = torch.channels_last
    m = C.ConvKxK(64, 64, 3, stride=1, padding=1).cuda().to(memory_format=cl)
    ref_w = m.weight.detach().double().clone().requires_grad_(True)
    opt = make_optimizer("sgd", m.parameters(), lr=0.0)
    x = torch.randn(4, 64, 28, 28, device="cuda").to(memory_format=cl)
    xg = x.detach().requires_grad_(True)
    xr = x.double().detach().requires_grad_(True)
    opt.zero_grad()
    y = m(xg)
    assert type(y.grad_fn).__name__.startswith("_ConvKxKFn")
    yr = F.conv2d(xr, ref_w, padding=1)
    g = torch.randn_like(yr)
    y.backward(g.float().to(memory_format=cl))
    yr.backward(g)
    for got, want in ((grad_of(m.weight), ref_w.grad), (xg.grad, xr.grad)):
        rel = float((got.double() - want).norm() / want.norm())
        assert rel < 1e-5, rel


@pytest.mark.gpu
def test_convkxk_c64_layer_uses_kernel_and_matches():
    """A 64-channel ConvKxK under a flat-gradient optimizer: weight gradient from the c64
    kernel into the fp32 flat buffer, input gradient as a forward conv."""
    from vodascheduler_amd.ops.optim import make_optimizer
    from vodascheduler_amd.utils.flat import grad_of

    torch.manual_seed(8)
    cl = torch.channels_last
    m = C.ConvKxK(64, 64, 3, stride=1, padding=1).cuda().to(memory_format=cl).bfloat16()
    ref_w = m.weight.detach().float().clone().requires_grad_(True)
    opt = make_optimizer("sgd", m.parameters(), lr=0.0)
    x = torch.randn(4, 64, 28, 28, device="cuda").bfloat16().to(memory_format=cl)
    xg = x.detach().requires_grad_(True)
    xr = x.float().detach().requires_grad_(True)
    opt.zero_grad()
    y = m(xg)
    assert type(y.grad_fn).__name__.startswith("_ConvKxKFn")
    yr = F.conv2d(xr, ref_w, padding=1)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16().to(memory_format=cl))
    yr.backward(g)
    for got, want in ((grad_of(m.weight), ref_w.grad), (xg.grad, xr.grad)):
        rel = float((got.float() - want).norm() / want.norm())
        assert rel < 1e-2, rel


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,stride", [(64, 64, 1), (128, 128, 1), (128, 128, 2), (256, 256, 2)])
def test_convkxk_fp32_layer_matches_fp64(cin, cout, stride):
    """fp32 (reference precision) ConvKxK: stride-1 input gradients run as forward
    convolutions (VODA_CONV_F32_FN), weight gradients on MIOpen -- against fp64 autograd."""
    torch.manual_seed(0)
    cl = torch.channels_last
    m = C.ConvKxK(cin, cout, 3, stride=stride, padding=1).cuda().to(memory_format=cl)
    x = torch.randn(2, cin, 14, 14, device="cuda").to(memory_format=cl).requires_grad_()
    y = m(x)
    if C.CONV_F32_FN and stride == 1:
        assert type(y.grad_fn).__name__.startswith("_ConvKxKFn")
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().double().requires_grad_()
    wr = m.weight.detach().double().requires_grad_()
    yr = F.conv2d(xr, wr, stride=stride, padding=1)
    yr.backward(dy.double())

    def rel(a, b):
        return float((a.double() - b).norm() / b.norm())

    assert rel(y, yr) < 1e-5 and rel(x.grad, xr.grad) < 1e-5 and rel(m.weight.grad, wr.grad) < 1e-5
