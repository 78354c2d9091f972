"""1x1-conv forward GEMM with BN statistics in the epilogue (csrc/hip/gemm_bnstats.hip,
ops/conv1x1.py) against fp32 PyTorch: the output, the partial sums / sums of squares, and the
ResNet bottleneck path (conv -> BN consuming the GEMM's statistics, forward and backward)."""
import pytest
import torch
import torch.nn.functional as F

from vodascheduler_amd.ops import _native as N
from vodascheduler_amd.ops import conv1x1 as C
from vodascheduler_amd.ops.batchnorm import STATS_ATTR, FusedBatchNorm2d

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,K,Nc", [(802816 // 64, 64, 256), (4096, 64, 512), (1000, 64, 256), (3136, 128, 512),
                                    (200, 128, 128), (77, 64, 256), (5000, 256, 64), (333, 256, 128)])
def test_gemm_bnstats_vs_fp32(M, K, Nc):
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(Nc, K, device="cuda") * 0.1).bfloat16()
    holder = C.StatsHolder()
    y = C.gemm_bnstats_2d(x, w, holder)
    assert y is not None and holder.stats is not None
    ref = x.float() @ w.float().t()
    torch.testing.assert_close(y.float(), ref, rtol=8e-3, atol=8e-3 * ref.abs().max().item())
    ws, G = holder.stats
    part = ws[: 2 * G * Nc].view(2, G, Nc).double().sum(1)
    rd = ref.double()
    # vs the unrounded product: within the bf16 rounding of the stored output (2^-8 relative
    # per element, bounded by the column's sum of magnitudes)
    tol1 = float((rd.abs().sum(0) * 2.0 ** -8).max())
    tol2 = float(((rd * rd).sum(0) * 2.0 ** -7).max())
    torch.testing.assert_close(part[0], rd.sum(0), rtol=0, atol=tol1)
    torch.testing.assert_close(part[1], (rd * rd).sum(0), rtol=0, atol=tol2)
    # the statistics are those of the STORED bf16 output (what BN normalises), up to fp32
    # summation order -- not of the unrounded accumulators
    yd = y.double()
    torch.testing.assert_close(part[0], yd.sum(0), rtol=1e-5, atol=1e-5 * M ** 0.5)
    torch.testing.assert_close(part[1], (yd * yd).sum(0), rtol=1e-5, atol=1e-5)


def test_gemm_bnstats_shape_gate():
    h = N.hip()
    assert h.gemm_bnstats_supported(1000, 256, 64) and h.gemm_bnstats_supported(1000, 128, 128)
    assert not h.gemm_bnstats_supported(1000, 64, 64)  # column tile is 256 at K = 64
    assert h.gemm_bnstats_supported(1000, 64, 256)
    assert not h.gemm_bnstats_supported(1000, 256, 256)  # K = 256: at most 2 column tiles
    assert not h.gemm_bnstats_supported(1000, 256, 512)


@pytest.mark.parametrize("cin,cout,stride,hw", [(64, 256, 1, 28), (128, 512, 1, 14), (128, 512, 2, 14),
                                                (256, 64, 1, 28)])
def test_conv_then_bn_uses_gemm_stats_and_matches(cin, cout, stride, hw, monkeypatch):
    """Conv1x1 -> FusedBatchNorm2d(+ReLU) in training: the BN takes the GEMM's statistics
    (no stats pass) and matches the fp32 composition, forward, running stats and grads."""
    torch.manual_seed(1)
    cl = torch.channels_last
    conv = C.Conv1x1(cin, cout, stride=stride).cuda().bfloat16().to(memory_format=cl)
    bn = FusedBatchNorm2d(cout, relu=True).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    x = torch.randn(8, cin, hw, hw, device="cuda").bfloat16().to(memory_format=cl).requires_grad_()
    seen = {}
    orig = C.gemm_bnstats_2d

    def spy(*a):
        r = orig(*a)
        seen["used"] = r is not None
        return r

    monkeypatch.setattr(C, "gemm_bnstats_2d", spy)
    y = conv(x)
    assert seen.get("used") and hasattr(y, STATS_ATTR)
    out = bn(y)
    assert not hasattr(y, STATS_ATTR)  # consumed
    # fp32 reference on the same bf16 operands
    xr = x.detach().float().requires_grad_()
    wr = conv.weight.detach().float().requires_grad_()
    yr = F.conv2d(xr, wr, stride=stride)
    ref_bn = torch.nn.BatchNorm2d(cout).cuda()
    ref_bn.load_state_dict({k: v for k, v in bn.state_dict().items() if k in ref_bn.state_dict()})
    ref_bn.running_mean.zero_(), ref_bn.running_var.fill_(1)
    outr = F.relu(ref_bn(yr.bfloat16().float()))
    torch.testing.assert_close(out.float(), outr, rtol=3e-2, atol=3e-2)
    bn.sync_batches_tracked()
    torch.testing.assert_close(bn.running_mean, ref_bn.running_mean, rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(bn.running_var, ref_bn.running_var, rtol=1e-2, atol=1e-3)
    g = torch.randn_like(outr)
    out.backward(g.bfloat16().to(memory_format=cl))
    outr.backward(g)
    for got, want in ((x.grad, xr.grad), (conv.weight.grad, wr.grad)):
        rel = float((got.float() - want).norm() / want.norm())
        assert rel < 3e-2, rel


@pytest.mark.parametrize("M,K,Nc", [(5000, 256, 64), (777, 64, 256), (3136, 128, 512)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_mfma_dgrad_matches_fp32(M, K, Nc, accumulate):
    """dX = dY . W on the MFMA GEMM (ops/conv1x1.mfma_dgrad): the [Cout][Cin] weight is
    transposed for the kernel; with ``acc2`` the result is added in place (beta = 1)."""
    torch.manual_seed(1)
    dy = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(K, Nc, device="cuda") * 0.1).bfloat16()   # [Cout = K][Cin = Nc]
    acc = torch.randn(M, Nc, device="cuda").bfloat16() if accumulate else None
    ref = dy.float() @ w.float() + (acc.float() if accumulate else 0.0)
    out = C.mfma_dgrad(dy, w, acc)
    assert out is not None
    if accumulate:
        assert out.data_ptr() == acc.data_ptr()
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
