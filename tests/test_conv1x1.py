"""1x1 convolutions as GEMMs (ops/conv1x1.py) against F.conv2d: forward, input gradient and
the weight gradient accumulated into the flat bf16 buffer by the split-K MFMA kernel."""
import copy

import pytest
import torch
import torch.nn.functional as F

from vodascheduler_amd.ops.conv1x1 import Conv1x1


def test_conv1x1_cpu_falls_back_to_conv2d():
    m = Conv1x1(16, 32, stride=2)
    x = torch.randn(2, 16, 8, 8)
    torch.testing.assert_close(m(x), F.conv2d(x, m.weight, stride=2))
    assert isinstance(m, torch.nn.Conv2d) and m.bias is None
    assert set(m.state_dict()) == {"weight"}


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / b.norm())


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,stride,hw", [(256, 64, 1, 14), (128, 512, 1, 7), (512, 1024, 2, 14),
                                               (1024, 256, 1, 7)])
def test_conv1x1_gemm_matches_conv2d(cin, cout, stride, hw):
    from vodascheduler_amd.ops.optim import make_optimizer

    torch.manual_seed(0)
    m = Conv1x1(cin, cout, stride=stride).cuda().to(memory_format=torch.channels_last).bfloat16()
    ref_w = m.weight.detach().float().clone().requires_grad_(True)
    opt = make_optimizer("sgd", m.parameters(), lr=0.0)  # flat grads: direct accumulation path
    x = torch.randn(4, cin, hw, hw, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    xr = x.float().detach().requires_grad_(True)
    xg = x.detach().requires_grad_(True)
    assert m._gemm_ok(xg)
    opt.zero_grad()
    y = m(xg)
    assert y.is_contiguous(memory_format=torch.channels_last)
    y_ref = F.conv2d(xr, ref_w, stride=stride)
    assert _rel(y, y_ref) < 1e-2
    g = torch.randn_like(y_ref)
    y.backward(g.bfloat16().to(memory_format=torch.channels_last))
    y_ref.backward(g)
    assert _rel(xg.grad, xr.grad) < 1e-2
    from vodascheduler_amd.utils.flat import grad_of

    assert grad_of(m.weight).dtype == torch.float32  # fp32 flat gradient of the bf16 weight
    assert _rel(grad_of(m.weight), ref_w.grad) < 1e-2
    # a second backward accumulates (beta = 1), as autograd does
    m(xg).backward(g.bfloat16().to(memory_format=torch.channels_last))
    assert _rel(grad_of(m.weight), 2 * ref_w.grad) < 1e-2


@pytest.mark.gpu
def test_resnet50_uses_gemm_path_and_trains():
    from vodascheduler_amd.models import get_workload, prepare_model
    from vodascheduler_amd.ops.optim import make_optimizer

    w = get_workload("resnet50")
    torch.manual_seed(0)
    m = prepare_model(w, torch.device("cuda", 0))
    opt = make_optimizer(w.optimizer, m.parameters(), **w.opt_kwargs)
    x, y = w.make_batch(8, torch.device("cuda", 0), None)
    x = x.to(memory_format=torch.channels_last)
    n_gemm = sum(1 for mod in m.modules() if isinstance(mod, Conv1x1) and mod.in_channels >= 128)
    assert n_gemm >= 20
    losses = []
    for _ in range(4):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = w.loss(m, (x, y))
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert all(torch.isfinite(torch.tensor(losses))) and losses[-1] < losses[0], losses


def test_grad_sink_handoff_cpu_semantics():
    from vodascheduler_amd.ops.conv1x1 import GradSink

    s = GradSink()
    assert s.take() is None
    g = torch.ones(2)
    s.put(g)
    assert s.take() is g and s.take() is None


def test_strided_grad_dense_is_the_zero_filled_scatter():
    """_StridedGrad (stride-2 downsample input gradient handed over subsampled) densifies to
    exactly the zero-filled channels_last scatter the consumer would otherwise receive."""
    from vodascheduler_amd.ops.conv1x1 import _StridedGrad

    g = torch.randn(2, 8, 3, 4).to(memory_format=torch.channels_last)
    d = _StridedGrad(g, 2, (2, 8, 6, 7)).dense()
    ref = torch.zeros(2, 8, 6, 7)
    ref[:, :, ::2, ::2] = g
    assert d.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(d, ref, atol=0, rtol=0)
    # the consumer's in-place form: full GEMM gradient + strided add == dense sum
    full = torch.randn(2, 8, 6, 7).to(memory_format=torch.channels_last)
    alt = full.clone()
    alt[:, :, ::2, ::2].add_(g)
    torch.testing.assert_close(alt, full + d, atol=0, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("downsample", [False, True])
def test_bottleneck_grad_sink_matches_autograd_sum(downsample, monkeypatch):
    """The shortcut gradient handed to conv1's dgrad GEMM (beta = 1) equals autograd's sum of
    the two input gradients, for the identity shortcut (bn3's residual gradient) and the
    stride-2 1x1 downsample (its scattered input gradient)."""
    import vodascheduler_amd.models.resnet as R
    from vodascheduler_amd.ops.batchnorm import FusedBatchNorm2d

    torch.manual_seed(0)
    cin, planes, stride = (512, 128, 2) if downsample else (256, 64, 1)
    down = None
    if downsample:
        down = torch.nn.Sequential(Conv1x1(cin, planes * 4, stride=stride), FusedBatchNorm2d(planes * 4))
    from vodascheduler_amd.models import cast_compute_weights_

    blk = R.Bottleneck(cin, planes, stride, down).cuda().to(memory_format=torch.channels_last)
    torch.nn.init.normal_(blk.bn3.weight)  # non-zero residual branch
    ref = copy.deepcopy(blk)  # fp32 reference (convolutions fall back to F.conv2d in fp32)
    cast_compute_weights_(blk)  # bf16 conv weights, fp32 BN parameters (as the trainer runs it)
    x = torch.randn(4, cin, 14, 14, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    g = torch.randn(4, planes * 4, 14 // stride, 14 // stride, device="cuda").bfloat16()
    g = g.to(memory_format=torch.channels_last)

    def run(model, xin, sink_on):
        monkeypatch.setattr(R, "USE_GRAD_SINK", sink_on)
        xi = xin.detach().clone().requires_grad_(True)
        model.zero_grad(set_to_none=True)
        y = model(xi)
        y.backward(g.to(y.dtype))
        return xi.grad.detach().float(), {n: p.grad.detach().float() for n, p in model.named_parameters()}

    # the bf16 forward is not bitwise reproducible across calls (stream-K GEMMs), so both bf16
    # runs are compared with the fp32 reference rather than with each other
    dx_r, pg_r = run(ref, x.float(), False)
    run(blk, x, False)  # first calls pick MIOpen / hipBLASLt algorithms
    dx0, pg0 = run(blk, x, False)
    dx1, pg1 = run(blk, x, True)
    e0, e1 = _rel(dx0, dx_r), _rel(dx1, dx_r)
    assert e1 < 0.2 and e1 < 1.1 * e0 + 5e-3, (e0, e1)  # bf16 vs fp32: e0 ~ 0.07 here
    for n in pg_r:
        e0, e1 = _rel(pg0[n], pg_r[n]), _rel(pg1[n], pg_r[n])
        assert e1 < 0.2 and e1 < 1.1 * e0 + 5e-3, (n, e0, e1)


def test_blas_wgrad_f32_rule():
    """fp32 1x1 weight gradients go to hipBLASLt only for short reductions into wide outputs
    (ResNet-50 stage 4 at bs 256), MIOpen keeps the rest (profiles/r4/blas_wgrad_f32_ab.jsonl)."""
    from vodascheduler_amd.ops.conv1x1 import blas_wgrad_f32_ok

    assert blas_wgrad_f32_ok(256 * 49, 2048, 512) and blas_wgrad_f32_ok(256 * 49, 512, 2048)
    assert blas_wgrad_f32_ok(256 * 49, 2048, 1024)          # stride-2 shortcut into stage 4
    assert not blas_wgrad_f32_ok(256 * 196, 1024, 256)      # stage 3: MIOpen 220 vs 558 us
    assert not blas_wgrad_f32_ok(256 * 49, 512, 512)        # narrow output
