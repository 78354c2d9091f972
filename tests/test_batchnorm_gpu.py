"""Fused BN(+residual)(+ReLU) HIP kernels vs an fp32 PyTorch reference (csrc/hip/batchnorm.hip)."""
import pytest
import torch
import torch.nn.functional as F

from vodascheduler_amd.ops.batchnorm import FusedBatchNorm2d, batch_norm_act

pytestmark = pytest.mark.gpu


def _ref(x, w, b, rm, rv, res, relu, mom, eps):
    y = F.batch_norm(x.float(), rm, rv, w, b, True, mom, eps)
    if res is not None:
        y = y + res.float()
    return F.relu(y) if relu else y


@pytest.mark.parametrize("shape", [(8, 64, 14, 14), (4, 80, 9, 9), (2, 256, 7, 5), (3, 2048, 3, 3), (2, 4096, 2, 3),
                                   (64, 64, 56, 56)])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False), (True, False)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_bn_act_fwd_bwd(shape, res, relu, dt):
    torch.manual_seed(0)
    dev = "cuda"
    C = shape[1]
    x = (torch.randn(shape, device=dev) * 2 + 0.5).to(dt).to(memory_format=torch.channels_last).requires_grad_()
    r = torch.randn(shape, device=dev).to(dt).to(memory_format=torch.channels_last).requires_grad_() if res else None
    w = (torch.rand(C, device=dev) + 0.5).requires_grad_()
    b = torch.randn(C, device=dev).requires_grad_()
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    rm2, rv2 = rm.clone(), rv.clone()
    y = batch_norm_act(x, w, b, rm, rv, True, 0.1, 1e-5, r, relu)
    assert y.is_contiguous(memory_format=torch.channels_last)
    xr = x.detach().float().requires_grad_()
    rr = r.detach().float().requires_grad_() if res else None
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    yr = _ref(xr, wr, br, rm2, rv2, rr, relu, 0.1, 1e-5)
    tol = 3e-2 if dt == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    torch.testing.assert_close(rm, rm2, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(rv, rv2, atol=1e-3, rtol=1e-3)
    dy = torch.randn(shape, device=dev).to(dt).to(memory_format=torch.channels_last)
    y.backward(dy)
    yr.backward(dy.float())
    gtol = 5e-2 if dt == torch.bfloat16 else 1e-3
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=gtol, rtol=gtol)
    M = x.numel() // C
    torch.testing.assert_close(w.grad, wr.grad, atol=gtol * M ** 0.5, rtol=gtol)
    torch.testing.assert_close(b.grad, br.grad, atol=gtol * M ** 0.5, rtol=gtol)
    if res:
        torch.testing.assert_close(r.grad.float(), rr.grad, atol=gtol, rtol=gtol)


@pytest.mark.parametrize("tuning", [(1, 2048, 1), (0, 1024, 0), (1, 64, 1), (1, 1024, 1), (2, 256, 0), (1, 256, 0),
                                    (1, 256, 2), (0, 64, 2), (2, 1024, 2)])
@pytest.mark.parametrize("shape", [(8, 64, 14, 14), (3, 2048, 3, 3), (16, 256, 28, 28)])
def test_bn_reduction_orders_agree(shape, tuning):
    """Every reduction walk (chunked / grid sweep, grid caps, unroll depths, buffer-descriptor
    tail clamping) gives the same statistics and gradients as the default."""
    from vodascheduler_amd.ops import _native

    h = _native.hip()
    saved = list(h.bn_get_tuning())
    torch.manual_seed(0)
    C = shape[1]
    x = (torch.randn(shape, device="cuda") + 0.3).to(torch.bfloat16).to(memory_format=torch.channels_last)
    r = torch.randn_like(x)
    dy = torch.randn_like(x)
    w = torch.rand(C, device="cuda") + 0.5
    b = torch.randn(C, device="cuda")

    def run():
        xi, ri = x.clone().requires_grad_(), r.clone().requires_grad_()
        wi, bi = w.clone().requires_grad_(), b.clone().requires_grad_()
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        y = batch_norm_act(xi, wi, bi, rm, rv, True, 0.1, 1e-5, ri, True)
        y.backward(dy)
        return [y.float(), rm, rv, xi.grad.float(), ri.grad.float(), wi.grad, bi.grad]

    try:
        h.bn_set_tuning(1, 1024, 0)
        base = run()
        h.bn_set_tuning(*tuning)
        other = run()
    finally:
        h.bn_set_tuning(*saved)
    M = x.numel() // C
    for i, (a, o) in enumerate(zip(base, other)):
        tol = 2e-2 * (M ** 0.5 if i >= 5 else 1)
        torch.testing.assert_close(o, a, atol=tol, rtol=2e-2, msg=f"output {i}")


def test_fused_bn_module_eval_and_autocast():
    torch.manual_seed(0)
    m = FusedBatchNorm2d(64, relu=True).cuda()
    ref = torch.nn.BatchNorm2d(64).cuda()
    ref.load_state_dict(m.state_dict())
    x = torch.randn(4, 64, 8, 8, device="cuda").to(memory_format=torch.channels_last)
    for _ in range(3):
        m(x)
        ref(x)
    torch.testing.assert_close(m.running_mean, ref.running_mean, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(m.running_var, ref.running_var, atol=1e-4, rtol=1e-4)
    assert int(m.state_dict()['num_batches_tracked']) == 3
    m.eval()
    ref.eval()
    torch.testing.assert_close(m(x), F.relu(ref(x)), atol=1e-5, rtol=1e-5)
    m.train()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        conv = torch.nn.Conv2d(64, 64, 1).cuda().to(memory_format=torch.channels_last)
        y = m(conv(x))
    assert y.dtype == torch.bfloat16


def test_resnet50_step_uses_fused_bn_kernels():
    from vodascheduler_amd.models import resnet50

    torch.manual_seed(0)
    m = resnet50().cuda().to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 64, 64, device="cuda").to(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(x)
    out.float().sum().backward()
    assert torch.isfinite(out.float()).all()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())


@pytest.mark.parametrize("shape,k,s,p", [((8, 64, 112, 112), 3, 2, 1), ((4, 96, 17, 17), 3, 2, 0), ((2, 64, 32, 32), 2, 2, 0),
                                         ((2, 8, 1, 5), 3, 2, 1), ((2, 16, 6, 6), 3, 2, 1),
                                         ((3, 8, 9, 7), 3, 1, 1)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_maxpool_nhwc_fwd_bwd(shape, k, s, p, dt):
    from vodascheduler_amd.ops.pool import max_pool2d

    torch.manual_seed(0)
    x = torch.randn(shape, device="cuda").to(dt).to(memory_format=torch.channels_last).requires_grad_()
    xr = x.detach().float().requires_grad_()
    y = max_pool2d(x, k, s, p)
    yr = F.max_pool2d(xr, k, s, p)
    torch.testing.assert_close(y.float(), yr, atol=0, rtol=0)
    dy = torch.randn_like(yr)
    y.backward(dy.to(dt))
    yr.backward(dy.to(dt).float())
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=1e-2 if dt == torch.bfloat16 else 1e-5, rtol=1e-2)


def test_bn_param_grads_accumulate_into_flat_buffer():
    from vodascheduler_amd.ops.optim import FusedSGD

    torch.manual_seed(0)
    a = FusedBatchNorm2d(64, relu=True).cuda()
    b = FusedBatchNorm2d(64, relu=True).cuda()
    b.load_state_dict(a.state_dict())
    FusedSGD(b.parameters(), lr=0.1)  # b's grads live in a flat buffer -> direct accumulation
    ready = []
    b.weight._voda_grad_ready = ready.append
    b.bias._voda_grad_ready = ready.append
    x = torch.randn(8, 64, 14, 14, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    for _ in range(2):
        for m in (a, b):
            xi = x.clone().requires_grad_()
            m(xi).float().square().sum().backward()
    assert len(ready) == 4
    torch.testing.assert_close(b.weight.grad, a.weight.grad, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(b.bias.grad, a.bias.grad, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("shape,k,s,p", [((4, 64, 112, 112), 3, 2, 1), ((3, 16, 17, 13), 3, 2, 1), ((2, 24, 9, 9), 3, 2, 0),
                                         ((2, 8, 7, 7), 3, 2, 1), ((2, 8, 1, 5), 3, 2, 1)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_bn_relu_maxpool_fused_matches_composition(shape, k, s, p, dt, monkeypatch):
    """maxpool(relu(bn(x))) on the fused stem kernels == the fp32 PyTorch composition:
    output, running statistics, input / gamma / beta gradients (the pooled gradient is
    gathered inside both BN backward passes)."""
    from vodascheduler_amd.ops import batchnorm
    from vodascheduler_amd.ops.batchnorm import FusedBNReLUMaxPool2d

    monkeypatch.setattr(batchnorm, "USE_FUSED_BN_POOL", True)

    torch.manual_seed(0)
    C = shape[1]
    m = FusedBNReLUMaxPool2d(C, k, s, p).cuda()
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    ref = torch.nn.BatchNorm2d(C).cuda()
    ref.load_state_dict({kk: v for kk, v in m.state_dict().items()})
    x = (torch.randn(shape, device="cuda") * 2 + 0.5).to(dt).to(memory_format=torch.channels_last)
    xi = x.clone().requires_grad_()
    y = m(xi)
    assert m._fused_ok(xi)
    xr = x.float().clone().requires_grad_()
    yr = F.max_pool2d(F.relu(ref(xr)), k, s, p)
    tol = 2e-2 if dt == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    torch.testing.assert_close(m.running_mean, ref.running_mean, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(m.running_var, ref.running_var, atol=1e-3, rtol=1e-3)
    dy = torch.randn_like(yr)
    y.backward(dy.to(dt))
    yr.backward(dy)
    M = x.numel() // C
    torch.testing.assert_close(xi.grad.float(), xr.grad, atol=5 * tol, rtol=5 * tol)
    torch.testing.assert_close(m.weight.grad, ref.weight.grad, atol=tol * M ** 0.5, rtol=tol)
    torch.testing.assert_close(m.bias.grad, ref.bias.grad, atol=tol * M ** 0.5, rtol=tol)


def test_bn_relu_maxpool_other_windows_compose(monkeypatch):
    """Windows other than 3x3/2 (not compiled into the fused kernels) take the composition."""
    from vodascheduler_amd.ops import batchnorm
    from vodascheduler_amd.ops.batchnorm import FusedBNReLUMaxPool2d

    monkeypatch.setattr(batchnorm, "USE_FUSED_BN_POOL", True)
    m = FusedBNReLUMaxPool2d(8, 2, 2, 0).cuda()
    x = torch.randn(2, 8, 8, 8, device="cuda").to(memory_format=torch.channels_last)
    assert not m._fused_ok(x)
    ref = torch.nn.BatchNorm2d(8).cuda()
    torch.testing.assert_close(m(x), F.max_pool2d(F.relu(ref(x)), 2, 2, 0), atol=1e-5, rtol=1e-5)


def test_bn_relu_maxpool_eval_path():
    from vodascheduler_amd.ops.batchnorm import FusedBNReLUMaxPool2d

    torch.manual_seed(0)
    m = FusedBNReLUMaxPool2d(16).cuda()
    x = torch.randn(2, 16, 12, 12, device="cuda").to(memory_format=torch.channels_last)
    m(x)
    m.eval()
    ref = torch.nn.BatchNorm2d(16).cuda().eval()
    ref.load_state_dict(m.state_dict())
    torch.testing.assert_close(m(x), F.max_pool2d(F.relu(ref(x)), 3, 2, 1), atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("shape", [(8, 64, 14, 14), (4, 256, 7, 5), (2, 2048, 3, 3), (32, 256, 28, 28)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bn_pair_matches_fp64_composition(shape, dt):
    """relu(bn(x) + bn2(x2)) as ONE dual-BN op (FusedBatchNorm2d.forward_pair, the ResNet
    downsample block's output) vs the fp64 composition of two BatchNorms: output, running
    statistics, and every gradient (x, x2, both gammas and betas)."""
    torch.manual_seed(1)
    dev = "cuda"
    C = shape[1]
    a = FusedBatchNorm2d(C, relu=True).to(dev)
    b = FusedBatchNorm2d(C).to(dev)
    with torch.no_grad():
        for m in (a, b):
            m.weight.uniform_(0.5, 1.5)
            m.bias.normal_()
    x = (torch.randn(shape, device=dev) * 2 + 0.5).to(dt).to(memory_format=torch.channels_last).requires_grad_()
    x2 = (torch.randn(shape, device=dev) - 0.3).to(dt).to(memory_format=torch.channels_last).requires_grad_()
    y = a.forward_pair(x, b, x2)
    assert y.is_contiguous(memory_format=torch.channels_last) and y.grad_fn.__class__.__name__ == "_BNAct2FnBackward"
    xr = x.detach().double().requires_grad_()
    x2r = x2.detach().double().requires_grad_()
    p = [t.detach().double().clone().requires_grad_() for t in (a.weight, a.bias, b.weight, b.bias)]
    rms = [torch.zeros(C, device=dev, dtype=torch.float64) for _ in range(2)]
    rvs = [torch.ones(C, device=dev, dtype=torch.float64) for _ in range(2)]
    yr = F.relu(F.batch_norm(xr, rms[0], rvs[0], p[0], p[1], True, 0.1, 1e-5)
                + F.batch_norm(x2r, rms[1], rvs[1], p[2], p[3], True, 0.1, 1e-5))
    tol = 3e-2 if dt == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.double(), yr, atol=tol, rtol=tol)
    for m, rm, rv in ((a, rms[0], rvs[0]), (b, rms[1], rvs[1])):
        torch.testing.assert_close(m.running_mean.double(), rm, atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(m.running_var.double(), rv, atol=1e-3, rtol=1e-3)
    dy = torch.randn(shape, device=dev).to(dt).to(memory_format=torch.channels_last)
    y.backward(dy)
    yr.backward(dy.double())
    gtol = 5e-2 if dt == torch.bfloat16 else 1e-3
    torch.testing.assert_close(x.grad.double(), xr.grad, atol=gtol, rtol=gtol)
    torch.testing.assert_close(x2.grad.double(), x2r.grad, atol=gtol, rtol=gtol)
    M = x.numel() // C
    for got, ref in zip((a.weight.grad, a.bias.grad, b.weight.grad, b.bias.grad), p):
        torch.testing.assert_close(got.double(), ref.grad, atol=gtol * M ** 0.5, rtol=gtol)


def test_resnet_downsample_block_pair_matches_two_bns(monkeypatch):
    """A ResNet-50 downsample bottleneck (fp32, channels_last, the GEMM / GradSink path) gives
    the same output and gradients with the dual-BN op as with bn3 + the shortcut BN apart."""
    from vodascheduler_amd.models import resnet as R

    torch.manual_seed(0)
    blk = R.Bottleneck(256, 128, stride=2, downsample=torch.nn.Sequential(
        R.Conv1x1(256, 512, stride=2), FusedBatchNorm2d(512))).cuda()
    with torch.no_grad():
        blk.bn3.weight.uniform_(0.5, 1.5)
    x = torch.randn(16, 256, 28, 28, device="cuda").to(memory_format=torch.channels_last)
    dy = torch.randn(16, 512, 14, 14, device="cuda").to(memory_format=torch.channels_last)
    outs = []
    for fuse in (True, False):
        monkeypatch.setattr(R, "FUSE_DOWNSAMPLE_BN", fuse)
        xi = x.clone().requires_grad_()
        for p_ in blk.parameters():
            p_.grad = None
        y = blk(xi)
        y.backward(dy)
        outs.append([y.detach(), xi.grad] + [p_.grad.clone() for p_ in blk.parameters()])
    for u, v in zip(*outs):
        torch.testing.assert_close(u, v, atol=1e-3, rtol=1e-3)  # fp32 summation order only
