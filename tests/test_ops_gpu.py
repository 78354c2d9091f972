"""Numerics of the hand-written HIP kernels vs plain PyTorch fp32 references (MI355X)."""
import math

import pytest
import torch

from vodascheduler_amd.ops import (FusedAdam, FusedLayerNorm, FusedRMSprop, FusedSGD, cast_scale_, layer_norm,
                                   masked_softmax, multi_tensor_copy_, reference_masked_softmax)
from vodascheduler_amd.ops import _native

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_native_extension_is_loaded():
    h = _native.hip()
    assert h.GPU_ARCH == "gfx950"
    assert torch.cuda.get_device_properties(0).gcnArchName.startswith("gfx950")


def _model_pair(seed=0):
    torch.manual_seed(seed)
    m1 = torch.nn.Sequential(torch.nn.Linear(33, 65), torch.nn.ReLU(), torch.nn.Linear(65, 7)).to(DEV)
    m2 = torch.nn.Sequential(torch.nn.Linear(33, 65), torch.nn.ReLU(), torch.nn.Linear(65, 7)).to(DEV)
    m2.load_state_dict(m1.state_dict())
    return m1, m2


def _run(m, opt, steps=5, seed=1):
    g = torch.Generator(device=DEV).manual_seed(seed)
    for _ in range(steps):
        x = torch.randn(16, 33, device=DEV, generator=g)
        opt.zero_grad()
        m(x).square().mean().backward()
        opt.step()


@pytest.mark.parametrize("kw", [dict(momentum=0.0), dict(momentum=0.9), dict(momentum=0.9, nesterov=True),
                                dict(momentum=0.9, weight_decay=1e-2, dampening=0.1)])
def test_fused_sgd_matches_torch(kw):
    m1, m2 = _model_pair()
    _run(m1, torch.optim.SGD(m1.parameters(), lr=0.1, **kw))
    _run(m2, FusedSGD(m2.parameters(), lr=0.1, **kw))
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("adamw", [False, True])
def test_fused_adam_matches_torch(adamw):
    m1, m2 = _model_pair()
    ref = (torch.optim.AdamW if adamw else torch.optim.Adam)(m1.parameters(), lr=1e-2, weight_decay=1e-2)
    _run(m1, ref)
    _run(m2, FusedAdam(m2.parameters(), lr=1e-2, weight_decay=1e-2, adamw=adamw))
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("kw", [dict(), dict(momentum=0.9), dict(centered=True, momentum=0.5)])
def test_fused_rmsprop_matches_torch(kw):
    m1, m2 = _model_pair()
    _run(m1, torch.optim.RMSprop(m1.parameters(), lr=1e-3, **kw))
    _run(m2, FusedRMSprop(m2.parameters(), lr=1e-3, **kw))
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


def test_fused_sgd_bf16_weights_and_grads():
    torch.manual_seed(0)
    m = torch.nn.Linear(128, 64).to(DEV).to(torch.bfloat16)
    opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9)
    master0 = opt.flat_groups[0].master.clone()
    x = torch.randn(8, 128, device=DEV, dtype=torch.bfloat16)
    opt.zero_grad()
    m(x).float().square().mean().backward()
    g = opt.flat_groups[0].grad.float().clone()
    opt.step()
    expect = master0 - 0.05 * g
    torch.testing.assert_close(opt.flat_groups[0].master, expect, rtol=1e-6, atol=1e-6)
    # bf16 model weights are the RNE cast of the fp32 master, written by the same kernel
    torch.testing.assert_close(opt.flat_groups[0].lowp, expect.to(torch.bfloat16), rtol=0, atol=0)


@pytest.mark.parametrize("n", [1, 3, 4, 1000, 65537, 1 << 22])
@pytest.mark.parametrize("sd,dd", [(torch.float32, torch.bfloat16), (torch.bfloat16, torch.float32),
                                   (torch.float32, torch.float16), (torch.float32, torch.float32)])
def test_cast_scale(n, sd, dd):
    x = torch.randn(n, device=DEV).to(sd)
    y = torch.empty(n, device=DEV, dtype=dd)
    cast_scale_(x, y, 0.125)
    torch.testing.assert_close(y, (x.float() * 0.125).to(dd), rtol=0, atol=0)


def test_multi_tensor_copy_roundtrip():
    ts = [torch.randn(s, device=DEV) for s in (1, 7, 64, 1000, 4097, 123456)] * 12  # > 64 tensors
    flat = torch.empty(sum(t.numel() for t in ts), device=DEV, dtype=torch.bfloat16)
    views = list(torch.split(flat, [t.numel() for t in ts]))
    multi_tensor_copy_(ts, views, scale=0.5)
    torch.testing.assert_close(flat, torch.cat(ts).mul(0.5).bfloat16(), rtol=0, atol=0)
    back = [torch.empty_like(t) for t in ts]
    multi_tensor_copy_(views, back, scale=2.0)
    for b, t in zip(back, ts):
        torch.testing.assert_close(b, t.bfloat16().float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("shape", [(10240, 256), (512, 768), (3, 5, 1024), (64, 4096), (7, 12)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layernorm_fwd_bwd(shape, dt):
    torch.manual_seed(0)
    n = shape[-1]
    x = torch.randn(shape, device=DEV).mul(3).add(1).to(dt).requires_grad_()
    w = torch.randn(n, device=DEV).requires_grad_()
    b = torch.randn(n, device=DEV).requires_grad_()
    y = layer_norm(x, w, b, 1e-5)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().clone().requires_grad_()
    br = b.detach().clone().requires_grad_()
    yr = torch.nn.functional.layer_norm(xr, (n,), wr, br, 1e-5)
    yr.backward(dy.float())
    tol = dict(rtol=2e-2, atol=3e-2) if dt == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)
    gt = dict(rtol=2e-2, atol=2e-1) if dt == torch.bfloat16 else dict(rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(w.grad, wr.grad, **gt)
    torch.testing.assert_close(b.grad, br.grad, **gt)


@pytest.mark.parametrize("shape", [(8192, 768), (10240, 256), (1000, 1024), (5, 12)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layernorm_bwd_4_and_8_waves_agree(shape, dt):
    """The 8-wave LayerNorm backward (the default for rows <= 1024) against the 4-wave one: dx
    bitwise (same per-row arithmetic), dgamma / dbeta to fp32 summation order."""
    from vodascheduler_amd.ops import _native

    h = _native.hip()
    torch.manual_seed(0)
    n = shape[-1]
    x = torch.randn(shape, device=DEV).mul(2).to(dt)
    w = torch.randn(n, device=DEV)
    b = torch.randn(n, device=DEV)
    dy = torch.randn(shape, device=DEV).to(dt)
    outs = []
    try:
        for waves in (4, 8):
            h.layernorm_set_bwd_waves(waves)
            xx, ww, bb = (t.clone().requires_grad_() for t in (x, w, b))
            layer_norm(xx, ww, bb, 1e-5).backward(dy)
            outs.append((xx.grad, ww.grad, bb.grad))
    finally:
        h.layernorm_set_bwd_waves(8)
    assert torch.equal(outs[0][0], outs[1][0])
    for a, c in zip(outs[0][1:], outs[1][1:]):
        torch.testing.assert_close(a, c, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("shape", [(512, 768), (3, 5, 1024), (7, 12)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layernorm_fused_residual(shape, dt):
    """LN(x + residual) in one kernel (the sum rounded to dt, as the unfused add would store
    it) vs an fp32 reference; both inputs receive the same gradient."""
    torch.manual_seed(0)
    n = shape[-1]
    x = torch.randn(shape, device=DEV).to(dt).requires_grad_()
    r = torch.randn(shape, device=DEV).mul(2).to(dt).requires_grad_()
    w = torch.randn(n, device=DEV).requires_grad_()
    b = torch.randn(n, device=DEV).requires_grad_()
    y = layer_norm(x, w, b, 1e-5, residual=r)
    dy = torch.randn_like(y)
    y.backward(dy)
    s = (x.detach() + r.detach()).float().requires_grad_()  # rounded sum, like the kernel's
    wr = w.detach().clone().requires_grad_()
    br = b.detach().clone().requires_grad_()
    yr = torch.nn.functional.layer_norm(s, (n,), wr, br, 1e-5)
    yr.backward(dy.float())
    tol = dict(rtol=2e-2, atol=3e-2) if dt == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(x.grad.float(), s.grad, **tol)
    torch.testing.assert_close(r.grad.float(), s.grad, **tol)
    gt = dict(rtol=2e-2, atol=2e-1) if dt == torch.bfloat16 else dict(rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(w.grad, wr.grad, **gt)
    torch.testing.assert_close(b.grad, br.grad, **gt)


@pytest.mark.parametrize("n", [8192 * 3072, 1000, 7, 8 * 257 + 5])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
def test_gelu_tanh_fwd_bwd(n, dt):
    """HIP tanh-GELU (csrc/hip/activation.hip) vs PyTorch's fp32 GELU, incl. the < 8 tail."""
    from vodascheduler_amd.ops.activation import gelu_tanh

    torch.manual_seed(0)
    h = torch.randn(n, device=DEV).mul(3).to(dt).requires_grad_()
    y = gelu_tanh(h)
    dy = torch.randn_like(y)
    y.backward(dy)
    hr = h.detach().float().requires_grad_()
    yr = torch.nn.functional.gelu(hr, approximate="tanh")
    yr.backward(dy.float())
    tol = dict(rtol=1e-5, atol=1e-5) if dt == torch.float32 else dict(rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(h.grad.float(), hr.grad, **tol)
    assert torch.isfinite(gelu_tanh(torch.tensor([-1e4, 1e4, -90.0, 90.0], device=DEV))).all()


def test_fused_layernorm_module_bf16_weights():
    ln = FusedLayerNorm(768).to(DEV).to(torch.bfloat16)
    x = torch.randn(4, 128, 768, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = ln(x)
    y.float().sum().backward()
    ref = torch.nn.functional.layer_norm(x.detach().float(), (768,))
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=3e-2)
    assert ln.weight.grad is not None and ln.weight.grad.dtype == torch.bfloat16


def test_fused_layernorm_flat_grads_accumulate_in_place():
    """gamma / beta gradients summed straight into the optimizer's flat fp32 buffer (one
    column-sum launch, beta = 1): equal to autograd's, and a second backward accumulates."""
    from vodascheduler_amd.ops.optim import make_optimizer

    torch.manual_seed(0)
    ln = FusedLayerNorm(768).to(DEV)
    torch.nn.init.normal_(ln.weight)
    torch.nn.init.normal_(ln.bias)
    opt = make_optimizer("adamw", ln.parameters(), lr=0.0)
    assert getattr(ln.weight, "_voda_flat_grad", False)
    x = torch.randn(4, 128, 768, device=DEV, dtype=torch.bfloat16)
    dy = torch.randn(4, 128, 768, device=DEV, dtype=torch.bfloat16)
    opt.zero_grad()
    ln(x).backward(dy)
    ref = torch.nn.LayerNorm(768).to(DEV)
    ref.load_state_dict(ln.state_dict())
    ref(x.float()).backward(dy.float())
    for got, want in ((ln.weight.grad, ref.weight.grad), (ln.bias.grad, ref.bias.grad)):
        torch.testing.assert_close(got, want, rtol=2e-2, atol=5e-2)
    ln(x).backward(dy)
    for got, want in ((ln.weight.grad, ref.weight.grad), (ln.bias.grad, ref.bias.grad)):
        torch.testing.assert_close(got, 2 * want, rtol=2e-2, atol=1e-1)


@pytest.mark.parametrize("B,H,Tq,S", [(512, 8, 20, 20), (4, 12, 128, 128), (2, 2, 7, 512), (1, 1, 3, 2048)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("causal", [False, True])
def test_masked_softmax(B, H, Tq, S, dt, causal):
    torch.manual_seed(0)
    x = torch.randn(B, H, Tq, S, device=DEV).mul(4).to(dt).requires_grad_()
    mask = (torch.rand(B, 1, 1, S, device=DEV) > 0.2).float()
    mask[..., 0] = 1
    scale = 1 / math.sqrt(64)
    y = masked_softmax(x, mask, causal, scale)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    yr = reference_masked_softmax(xr, mask, causal, scale)
    yr.backward(dy.float())
    tol = dict(rtol=2e-2, atol=1e-2) if dt == torch.bfloat16 else dict(rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)


@pytest.mark.parametrize("M,Nc,dt,odt", [(8192, 768, torch.bfloat16, torch.bfloat16), (1000, 3072, torch.bfloat16,
                                                                                       torch.float32),
                                        (37, 2304, torch.float32, torch.float32), (5, 8, torch.float16, torch.float32),
                                        (300, 4096, torch.bfloat16, torch.float32)])
def test_colsum_accumulate(M, Nc, dt, odt):
    from vodascheduler_amd.ops.dense import colsum_accumulate_

    torch.manual_seed(0)
    x = torch.randn(M, Nc, device="cuda").to(dt)
    out = torch.randn(Nc, device="cuda").to(odt)
    ref = out.float() + x.float().sum(0)
    colsum_accumulate_(x, out)
    tol = 2e-2 * max(1.0, M ** 0.5) if odt == torch.bfloat16 else 1e-3 * max(1.0, M ** 0.5)
    torch.testing.assert_close(out.float(), ref, atol=tol, rtol=1e-2)


def test_fused_linear_bf16_flat_grads_gpu():
    from vodascheduler_amd.models import cast_compute_weights_
    from vodascheduler_amd.ops.dense import FusedLinear
    from vodascheduler_amd.ops.optim import FusedAdamW

    torch.manual_seed(0)
    ref = torch.nn.Linear(768, 3072).cuda()
    m = FusedLinear(768, 3072).cuda()
    m.load_state_dict(ref.state_dict())
    cast_compute_weights_(m)
    FusedAdamW(m.parameters(), lr=1e-3)
    x = torch.randn(8, 128, 768, device="cuda")
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
        yr = ref(x)
    g = torch.randn_like(yr.float())
    y.float().backward(g)
    yr.float().backward(g)
    torch.testing.assert_close(y.float(), yr.float(), atol=5e-2, rtol=5e-2)
    from vodascheduler_amd.utils.flat import grad_of

    assert m.weight.grad is None and grad_of(m.weight).dtype == torch.float32  # fp32 flat gradient
    # loose: against the stock layer (its own autocast GEMM rounds dW to bf16)
    torch.testing.assert_close(grad_of(m.weight), ref.weight.grad, atol=0.5, rtol=5e-2)
    torch.testing.assert_close(grad_of(m.bias), ref.bias.grad, atol=0.5, rtol=5e-2)
    # tight: against the exact (fp64) product of the bf16 operands the kernel consumes -- the
    # MFMA kernel accumulates in fp32 and rounds once, so a wrong tile / k-step / lane map
    # (errors of the gradient's own magnitude, ~30 here) cannot hide under the tolerance
    gq = g.bfloat16().double().reshape(-1, 3072)
    xq = x.bfloat16().double().reshape(-1, 768)
    torch.testing.assert_close(grad_of(m.weight).double(), gq.t() @ xq, rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(grad_of(m.bias).double(), gq.sum(0), rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("opt_name", ["adamw", "sgd"])
def test_overlapped_per_bucket_optimizer_matches_plain_step(opt_name):
    """ElasticDDP(overlap_optimizer=True): per-bucket updates on the comm stream during
    backward give bitwise the same weights as one optimizer pass after backward."""
    from vodascheduler_amd.models import cast_compute_weights_
    from vodascheduler_amd.ops.dense import FusedLinear
    from vodascheduler_amd.ops.layernorm import FusedLayerNorm
    from vodascheduler_amd.ops.optim import make_optimizer
    from vodascheduler_amd.parallel.ddp import ElasticDDP

    def build():
        torch.manual_seed(0)
        layers = []
        for _ in range(6):
            layers += [FusedLinear(512, 512), FusedLayerNorm(512)]
        return cast_compute_weights_(torch.nn.Sequential(*layers).cuda())

    kw = dict(lr=1e-3, weight_decay=0.01) if opt_name == "adamw" else dict(lr=0.05, momentum=0.9)
    runs = []
    for overlap in (False, True):
        m = build()
        opt = make_optimizer(opt_name, m.parameters(), **kw)
        ddp = ElasticDDP(m, None, opt, bucket_cap_mb=1.0, first_bucket_mb=0.5, overlap_optimizer=overlap)
        assert len(ddp.buckets) >= 4
        x = torch.randn(1024, 512, device="cuda").bfloat16()
        for _ in range(3):
            ddp.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
                loss = m(x).float().square().mean()
            loss.backward()
            ddp.step()
        torch.cuda.synchronize()
        runs.append([t.clone() for t in opt.flat_state_tensors()])
    for a, b in zip(*runs):
        assert torch.equal(a, b)
