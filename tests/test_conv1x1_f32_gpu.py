"""fp32 1x1-convolution GEMMs on the f32 MFMA (csrc/hip/conv1x1_f32.hip) against fp64 PyTorch
references of the same ops: the forward GEMM with its BN statistics epilogue (and the
accumulating form used for input gradients), the split-K weight gradient in every wave
layout, and the Conv1x1 module's fp32 GEMM path end to end (VERDICT r3 Next #4)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _h():
    from vodascheduler_amd.ops import _native as N

    return N.hip(), N


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("M,N,K", [(1000, 256, 64), (4096, 512, 64), (777, 128, 128), (2048, 256, 128),
                                   (300, 64, 256), (5000, 128, 256)])
def test_gemm_f32_stats_matches_fp64(M, N, K):
    h, Nn = _h()
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") * 0.1
    assert h.gemm_f32_stats_supported(M, N, K)
    G = h.gemm_f32_stats_groups(M, N, K)
    y = torch.full((M, N), float("nan"), device="cuda")
    part = torch.empty(2 * G * N, device="cuda")
    h.gemm_f32_stats(x.data_ptr(), w.data_ptr(), y.data_ptr(), part.data_ptr(), M, N, K, G, Nn.stream_of(x), False, False)
    ref = x.double() @ w.double().t()
    assert _rel(y, ref) < 2e-6
    s1 = part[:G * N].view(G, N).double().sum(0)
    s2 = part[G * N:].view(G, N).double().sum(0)
    assert _rel(s1, ref.sum(0)) < 1e-5 and _rel(s2, (ref * ref).sum(0)) < 1e-5
    # accumulate form (input gradient into a tensor that already holds the shortcut's)
    y0 = torch.randn(M, N, device="cuda")
    y2 = y0.clone()
    h.gemm_f32_stats(x.data_ptr(), w.data_ptr(), y2.data_ptr(), 0, M, N, K, G, Nn.stream_of(x), True, False)
    assert _rel(y2, y0.double() + ref) < 2e-6
    # W handed over as [K][N] (the input-gradient form: no transposed copy)
    wkn = w.t().contiguous()
    y3 = torch.full((M, N), float("nan"), device="cuda")
    h.gemm_f32_stats(x.data_ptr(), wkn.data_ptr(), y3.data_ptr(), 0, M, N, K, G, Nn.stream_of(x), False, True)
    assert torch.equal(y3, y)


@pytest.mark.parametrize("cin,cout,stride,hw", [(64, 256, 1, 14), (256, 64, 1, 9), (128, 512, 1, 7),
                                               (512, 1024, 2, 14), (1024, 256, 1, 7), (256, 512, 2, 8),
                                               (512, 2048, 1, 7), (1024, 2048, 2, 14)])
def test_conv1x1_fp32_gemm_path_matches_fp64(cin, cout, stride, hw):
    """fp32 channels_last Conv1x1 on the GEMM path (own forward / input gradient where K is 64 /
    128 / 256, hipBLASLt elsewhere, weight gradient folded into the fp32 flat gradient -- from
    MIOpen, or from one beta = 1 hipBLASLt GEMM for the wide stage-4 outputs)."""
    from vodascheduler_amd.ops.conv1x1 import Conv1x1
    from vodascheduler_amd.ops.optim import make_optimizer
    from vodascheduler_amd.utils.flat import grad_of

    torch.manual_seed(0)
    m = Conv1x1(cin, cout, stride=stride).cuda().to(memory_format=torch.channels_last)
    ref_w = m.weight.detach().double().clone().requires_grad_(True)
    opt = make_optimizer("sgd", m.parameters(), lr=0.0)
    x = torch.randn(4, cin, hw, hw, device="cuda").to(memory_format=torch.channels_last)
    xg = x.detach().requires_grad_(True)
    xr = x.double().detach().requires_grad_(True)
    assert m._gemm_ok(xg)
    opt.zero_grad()
    y = m(xg)
    assert "Conv1x1Fn" in type(y.grad_fn).__name__
    y_ref = F.conv2d(xr, ref_w, stride=stride)
    assert _rel(y, y_ref) < 1e-5
    g = torch.randn_like(y_ref)
    y.backward(g.float().to(memory_format=torch.channels_last))
    y_ref.backward(g)
    assert _rel(xg.grad, xr.grad) < 1e-5
    assert grad_of(m.weight).dtype == torch.float32
    assert _rel(grad_of(m.weight), ref_w.grad) < 1e-5
    m(xg).backward(g.float().to(memory_format=torch.channels_last))   # accumulates (beta = 1)
    assert _rel(grad_of(m.weight), 2 * ref_w.grad) < 1e-5


def test_conv1x1_fp32_bn_statistics_attached():
    """Training-mode fp32 Conv1x1 -> FusedBatchNorm2d: the statistics come from the GEMM
    epilogue and the BN output equals conv2d + batch_norm in fp64."""
    from vodascheduler_amd.ops.batchnorm import FusedBatchNorm2d
    from vodascheduler_amd.ops.conv1x1 import Conv1x1

    torch.manual_seed(1)
    conv = Conv1x1(128, 512).cuda().to(memory_format=torch.channels_last)
    bn = FusedBatchNorm2d(512, relu=True).cuda()
    conv.train(), bn.train()
    x = torch.randn(8, 128, 14, 14, device="cuda").to(memory_format=torch.channels_last).requires_grad_(True)
    assert conv._stats_ok(x)
    y = conv(x)
    from vodascheduler_amd.ops.batchnorm import STATS_ATTR

    assert getattr(y, STATS_ATTR, None) is not None   # statistics from the GEMM epilogue
    z = bn(y)
    yr = F.conv2d(x.double(), conv.weight.double())
    zr = F.relu(F.batch_norm(yr, None, None, bn.weight.double(), bn.bias.double(), training=True, eps=bn.eps))
    assert _rel(z, zr) < 1e-5


def _bits(m: torch.Tensor) -> torch.Tensor:
    """[M, C] bool -> the BN forward's 1-bit ReLU mask ([M * C / 8] bytes, bit k of byte (r, g) =
    channel 8 g + k)."""
    M, C = m.shape
    w = (m.view(M, C // 8, 8).to(torch.int32) << torch.arange(8, device=m.device, dtype=torch.int32)).sum(-1)
    return w.to(torch.uint8).reshape(-1).contiguous()


@pytest.mark.parametrize("M,K,N", [(4096, 64, 256), (3000, 128, 512), (1111, 256, 1024), (50176, 64, 256)])
@pytest.mark.parametrize("nsums", [0, 2, 3])
def test_fused_dgrad_bn_matches_fp64(M, K, N, nsums):
    """gemm_f32_dgrad_bn: dX = dY . W + g * bits(cmask) and the downstream BN's backward sums
    (sum h, sum h*y3 [, sum h*y_ds], h = dX * bits(smask)) vs fp64; ragged M exercises the
    buffer-clamped tail rows."""
    from vodascheduler_amd.ops import _native

    h = _native.hip()
    torch.manual_seed(M + K + nsums)
    dev = "cuda"
    dy = torch.randn(M, K, device=dev)
    w = torch.randn(K, N, device=dev) / K ** 0.5
    g = torch.randn(M, N, device=dev)
    cm = torch.rand(M, N, device=dev) > 0.4
    sm = torch.rand(M, N, device=dev) > 0.5
    y3 = torch.randn(M, N, device=dev)
    yd = torch.randn(M, N, device=dev)
    G = h.gemm_f32_dgrad_bn_groups(M, N, K, nsums)
    out = torch.empty(M, N, device=dev)
    part = torch.empty(max(1, nsums * G * N), device=dev)
    cmb, smb = _bits(cm), _bits(sm)
    h.gemm_f32_dgrad_bn(dy.data_ptr(), w.data_ptr(), out.data_ptr(), g.data_ptr(), cmb.data_ptr(),
                        smb.data_ptr() if nsums else 0, y3.data_ptr() if nsums else 0,
                        yd.data_ptr() if nsums == 3 else 0, part.data_ptr() if nsums else 0, M, N, K, G, nsums,
                        torch.cuda.current_stream().cuda_stream)
    ref = dy.double() @ w.double() + g.double() * cm
    torch.testing.assert_close(out.double(), ref, atol=1e-4, rtol=1e-5)
    if nsums:
        hh = ref * sm
        want = [hh.sum(0), (hh * y3.double()).sum(0), (hh * yd.double()).sum(0)][:nsums]
        got = part[:nsums * G * N].view(nsums, G, N).double().sum(1)
        for j in range(nsums):
            torch.testing.assert_close(got[j], want[j], atol=2e-3 * M ** 0.5, rtol=1e-4)


@pytest.mark.parametrize("fuse_pair", [True, False])
def test_resnet_stage_fused_dgrad_bn_matches_unfused(monkeypatch, fuse_pair):
    """A ResNet-50 stage (downsample block + two identity blocks, fp32 channels_last): with the
    fused input gradient + BN handoff the output, the input gradient and every parameter
    gradient equal the unfused path's (hipBLASLt beta = 1 + BN reduce passes) to fp32 order."""
    from vodascheduler_amd.models import resnet as R
    from vodascheduler_amd.ops import conv1x1 as C
    from vodascheduler_amd.ops.batchnorm import FusedBatchNorm2d

    monkeypatch.setattr(R, "FUSE_DOWNSAMPLE_BN", fuse_pair)
    torch.manual_seed(0)
    blocks = torch.nn.Sequential(
        R.Bottleneck(256, 128, stride=2, downsample=torch.nn.Sequential(R.Conv1x1(256, 512, stride=2),
                                                                        FusedBatchNorm2d(512))),
        R.Bottleneck(512, 128), R.Bottleneck(512, 128)).cuda()
    with torch.no_grad():
        for b in blocks:
            b.bn3.weight.uniform_(0.5, 1.5)
    x = torch.randn(8, 256, 28, 28, device="cuda").to(memory_format=torch.channels_last)
    dy = torch.randn(8, 512, 14, 14, device="cuda").to(memory_format=torch.channels_last)
    from vodascheduler_amd.ops import batchnorm as B

    calls = {"kernel": 0, "sums": 0}
    real_fused, real_take = C.fused_dgrad_bn, B.BwdHandoff.take

    def fused(*a):
        r = real_fused(*a)
        calls["kernel"] += r is not None
        return r

    def take(self, dy):
        r = real_take(self, dy)
        calls["sums"] += r is not None
        return r

    monkeypatch.setattr(C, "fused_dgrad_bn", fused)
    monkeypatch.setattr(B.BwdHandoff, "take", take)
    outs = []
    for fused_on in (True, False):
        monkeypatch.setattr(C, "USE_FUSED_DGRAD_BN", fused_on)
        xi = x.clone().requires_grad_()
        for p_ in blocks.parameters():
            p_.grad = None
        y = blocks(xi)
        y.backward(dy)
        outs.append([y.detach(), xi.grad] + [p_.grad.clone() for p_ in blocks.parameters()])
        if fused_on:  # both identity blocks ran the fused kernel; blocks 1 and 2's bn3 took its sums
            assert calls == {"kernel": 2, "sums": 2}, calls
    # relative Frobenius error per tensor: MIOpen's split-K convolutions accumulate with atomics,
    # so two runs of the SAME path already differ in the last bits, and the BN backward's
    # cancellations (sum g*x - mean * sum g) amplify any summation-order change elementwise;
    # the exact semantics are pinned by test_fused_dgrad_bn_matches_fp64
    names = ["y", "x.grad"] + [n for n, _ in blocks.named_parameters()]
    rel = [(nm, float((u - v).norm() / v.norm().clamp_min(1e-12))) for nm, u, v in zip(names, *outs)]
    # observed 0.3-2.6e-4 between the paths over repeated runs; a wrong mask, a missing
    # shortcut term or stale sums give O(1) errors
    bad = [(nm, e) for nm, e in rel if e > 1e-3]
    assert not bad, bad
