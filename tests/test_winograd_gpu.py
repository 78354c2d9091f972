"""Winograd F(2x2, 3x3) fp32 convolution (csrc/hip/winograd_f32.hip) against an fp64 PyTorch
reference: ResNet-50 3x3 shapes, odd sizes (ragged last tile), tile counts off the 32-tile
workgroup, channel counts that are multiples of 32, channels_last and contiguous filters."""
import pytest
import torch
import torch.nn.functional as F

from vodascheduler_amd.ops import winograd as Wg

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[(False, False, True), (True, False, False), (True, False, True), (True, True, True)],
                ids=["f32mfma", "bf16x3-pairs", "bf16x3", "bf16x3-wide"])
def sx(request, monkeypatch):
    """The tile-GEMM paths: the f32 MFMA, the exact 3-way bf16 split (Wg.USE_SX) at 32 output
    channels per workgroup (position pairs or one position at a time, Wg.ONEPOS), and the split at
    64 (Wg.USE_WIDE, Cout % 64 == 0)."""
    monkeypatch.setattr(Wg, "USE_SX", request.param[0])
    monkeypatch.setattr(Wg, "USE_WIDE", request.param[1])
    monkeypatch.setattr(Wg, "ONEPOS", request.param[2])
    monkeypatch.setattr(Wg, "WIDE_MAX_C", 1 << 20)  # the wide kernel on every covered shape
    return request.param[0]


@pytest.mark.parametrize("n,c,co,h,w", [(2, 64, 64, 56, 56), (3, 128, 96, 28, 28), (4, 256, 256, 14, 14),
                                        (5, 512, 512, 7, 7), (1, 32, 32, 5, 9), (3, 64, 32, 1, 1),
                                        (3, 96, 128, 9, 7), (1, 32, 64, 3, 3)])
@pytest.mark.parametrize("wcl", [True, False])
def test_wino_f23_matches_fp64(n, c, co, h, w, wcl, sx):
    torch.manual_seed(c + h)
    x = torch.randn(n, c, h, w, device="cuda").contiguous(memory_format=torch.channels_last)
    wt = torch.randn(co, c, 3, 3, device="cuda") / (3 * c ** 0.5)
    if wcl:
        wt = wt.contiguous(memory_format=torch.channels_last)
    assert Wg.supported(x, wt)
    y = Wg.conv3x3_wino(x, wt)
    ref = F.conv2d(x.double(), wt.double(), None, 1, 1)
    rel = ((y.double() - ref).norm() / ref.norm()).item()
    assert rel < 2e-6, rel
    assert (y.double() - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("n,c,co,h", [(2, 64, 64, 56), (3, 256, 128, 14), (2, 512, 512, 7), (1, 64, 32, 5)])
def test_wino_f23_input_gradient_matches_fp64(n, c, co, h, sx):
    """flip mode: dX of a 3x3 stride-1 pad-1 layer with filter [co][c] from dY [n][co][h][h]."""
    torch.manual_seed(c + h)
    dy = torch.randn(n, co, h, h, device="cuda").contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(co, c, 3, 3, device="cuda") / (3 * c ** 0.5)).contiguous(memory_format=torch.channels_last)
    assert Wg.supported(dy, wt, flip=True)
    dx = Wg.conv3x3_wino(dy, wt, flip=True)
    ref = torch.nn.grad.conv2d_input((n, c, h, h), wt.double(), dy.double(), stride=1, padding=1)
    rel = ((dx.double() - ref).norm() / ref.norm()).item()
    assert rel < 2e-6, rel


@pytest.mark.parametrize("n,c,co,h", [(4, 64, 64, 56), (3, 256, 256, 14), (5, 512, 512, 7), (2, 32, 64, 9)])
def test_wino_f23_bn_partials(n, c, co, h, sx):
    """The epilogue's per-workgroup BN partial sums add up to the column sums of y and y^2."""
    from vodascheduler_amd.ops.conv1x1 import StatsHolder

    torch.manual_seed(h)
    x = torch.randn(n, c, h, h, device="cuda").contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(co, c, 3, 3, device="cuda") / (3 * c ** 0.5)).contiguous(memory_format=torch.channels_last)
    hd = StatsHolder()
    y = Wg.conv3x3_wino(x, wt, holder=hd)
    ws, G = hd.stats
    part = ws[: 2 * G * co].view(2, G, co).double().sum(1)
    yd = y.double().permute(0, 2, 3, 1).reshape(-1, co)
    torch.testing.assert_close(part[0], yd.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(part[1], (yd * yd).sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("n,c,h", [(2, 128, 28), (2, 512, 7)])
def test_wino_sx_error_no_worse_than_f32_mfma(n, c, h):
    """The split-bf16 tile GEMMs are as accurate as the f32 MFMA ones (both vs fp64), also for
    operands whose magnitudes span 2^+-20."""
    torch.manual_seed(c)
    x = torch.randn(n, c, h, h, device="cuda")
    x = (x * torch.exp2(torch.randint(-20, 21, x.shape, device="cuda").float())).contiguous(
        memory_format=torch.channels_last)
    wt = (torch.randn(c, c, 3, 3, device="cuda") / (3 * c ** 0.5)).contiguous(memory_format=torch.channels_last)
    ref = F.conv2d(x.double(), wt.double(), None, 1, 1)
    bound = F.conv2d(x.double().abs(), wt.double().abs(), None, 1, 1) + 1e-30
    err = {}
    for sxv in (False, True):
        y = Wg.conv3x3_wino(x, wt, u=Wg.filter_transform(wt, sx=sxv))
        err[sxv] = ((y.double() - ref).abs() / bound).max().item()
    assert err[True] <= 1.5 * err[False] + 1e-7, err
    u = Wg.filter_transform(wt, sx=True)
    assert u.dtype == torch.bfloat16 and u.numel() == 48 * c * c


def test_resnet_fp32_step_with_winograd_matches_miopen(monkeypatch):
    """A small fp32 ResNet-50 training step with the Winograd 3x3 layers (and their BN statistics)
    vs the same step on MIOpen: loss and every gradient agree to fp32 rounding."""
    from vodascheduler_amd.models.resnet import resnet50
    from vodascheduler_amd.ops import conv3x3 as C3

    torch.manual_seed(0)
    m = resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    tgt = torch.randint(0, 10, (4,), device="cuda")

    def run(wino):
        monkeypatch.setattr(C3, "USE_WINOGRAD", wino)
        m.zero_grad(set_to_none=True)
        loss = torch.nn.functional.cross_entropy(m(x), tgt)
        loss.backward()
        return [loss.detach()] + [p.grad.clone() for p in m.parameters()]

    a, b = run(True), run(False)
    for i, (u, v) in enumerate(zip(a, b)):
        rel = ((u.double() - v.double()).norm() / (v.double().norm() + 1e-12)).item()
        assert rel < 1e-3, f"tensor {i}: {rel}"
