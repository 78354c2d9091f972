"""CPU reference paths of the fused ops (the same flat-buffer math the HIP kernels run)."""
import copy
import pytest
import torch

from vodascheduler_amd.ops import (FusedAdam, FusedRMSprop, FusedSGD, cast_scale_, layer_norm, make_optimizer,
                                   masked_softmax, multi_tensor_copy_, reference_masked_softmax)
from vodascheduler_amd.utils.flat import FlatGroup


def _pair():
    torch.manual_seed(0)
    a = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.Flatten(), torch.nn.Linear(8 * 6 * 6, 5))
    b = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.Flatten(), torch.nn.Linear(8 * 6 * 6, 5))
    b.load_state_dict(a.state_dict())
    return a, b


def _train(m, opt, steps=4):
    g = torch.Generator().manual_seed(3)
    for _ in range(steps):
        x = torch.randn(4, 3, 8, 8, generator=g)
        opt.zero_grad()
        m(x).square().mean().backward()
        opt.step()


@pytest.mark.parametrize("ours,ref,kw", [
    (FusedSGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9, weight_decay=1e-3)),
    (FusedSGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9, nesterov=True)),
    (FusedSGD, torch.optim.SGD, dict(lr=0.1)),
    (FusedAdam, torch.optim.Adam, dict(lr=1e-2, weight_decay=1e-3)),
    (FusedRMSprop, torch.optim.RMSprop, dict(lr=1e-3, momentum=0.9, centered=True)),
])
def test_cpu_optimizers_match_torch(ours, ref, kw):
    a, b = _pair()
    _train(a, ref(a.parameters(), **kw))
    _train(b, ours(b.parameters(), **kw))
    for x, y in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)


def test_flat_group_keeps_channels_last_and_views():
    conv = torch.nn.Conv2d(4, 8, 3).to(memory_format=torch.channels_last)
    st = conv.weight.stride()
    fg = FlatGroup(conv.parameters())
    assert conv.weight.stride() == st
    assert conv.weight.data_ptr() == fg.master.data_ptr()
    out = conv(torch.randn(2, 4, 5, 5).to(memory_format=torch.channels_last))
    out.sum().backward()
    assert conv.weight.grad.data_ptr() == fg.grad.data_ptr()
    assert fg.grad.abs().sum() > 0
    fg.zero_grad()
    assert fg.grad.abs().sum() == 0


def test_optimizer_state_dict_roundtrip():
    a, b = _pair()
    oa = make_optimizer("adam", a.parameters(), lr=1e-2)
    _train(a, oa)
    ob = make_optimizer("adam", b.parameters(), lr=1e-2)
    ob.load_state_dict(oa.state_dict())
    for x, y in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(x, y)
    _train(a, oa, 2)
    _train(b, ob, 2)
    for x, y in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(x, y)


def test_cpu_cast_and_multi_copy():
    x = torch.randn(100)
    y = torch.empty(100, dtype=torch.bfloat16)
    cast_scale_(x, y, 0.5)
    torch.testing.assert_close(y, (x * 0.5).bfloat16())
    ts = [torch.randn(5), torch.randn(7)]
    out = [torch.empty(5), torch.empty(7)]
    multi_tensor_copy_(ts, out, 2.0)
    torch.testing.assert_close(out[1], ts[1] * 2)


def test_cpu_layernorm_residual_and_gelu_fallbacks():
    """``layer_norm(x, residual=r)`` == LN(x + r) with both gradients; CPU tanh-GELU."""
    from vodascheduler_amd.ops.activation import gelu_tanh

    x = torch.randn(3, 16, requires_grad=True)
    r = torch.randn(3, 16, requires_grad=True)
    layer_norm(x, residual=r).square().sum().backward()
    xs = (x.detach() + r.detach()).requires_grad_()
    torch.nn.functional.layer_norm(xs, (16,)).square().sum().backward()
    torch.testing.assert_close(x.grad, xs.grad)
    torch.testing.assert_close(r.grad, xs.grad)
    h = torch.randn(100)
    torch.testing.assert_close(gelu_tanh(h), torch.nn.functional.gelu(h, approximate="tanh"))


def test_cpu_layernorm_and_softmax_reference():
    x = torch.randn(3, 16)
    torch.testing.assert_close(layer_norm(x), torch.nn.functional.layer_norm(x, (16,)))
    s = torch.randn(2, 2, 4, 4)
    y = masked_softmax(s, causal=True)
    assert torch.allclose(y.sum(-1), torch.ones(2, 2, 4))
    assert y[0, 0, 0, 1:].abs().max() < 1e-6
    torch.testing.assert_close(y, reference_masked_softmax(s, None, True))


def test_fused_bn_module_cpu_matches_reference():
    import torch.nn.functional as F

    from vodascheduler_amd.ops.batchnorm import FusedBatchNorm2d

    torch.manual_seed(0)
    m = FusedBatchNorm2d(16, relu=True)
    ref = torch.nn.BatchNorm2d(16)
    x = torch.randn(4, 16, 5, 5)
    r = torch.randn(4, 16, 5, 5)
    torch.testing.assert_close(m(x, r), F.relu(ref(x) + r))
    torch.testing.assert_close(m.running_var, ref.running_var)


def test_optimizer_splits_param_groups_by_dtype():
    from vodascheduler_amd.models import cast_compute_weights_
    from vodascheduler_amd.models.transformer import BertBase
    from vodascheduler_amd.ops.optim import FusedAdamW

    m = BertBase(vocab=100, seq_len=8, d_model=32, heads=2, d_ff=64, layers=1)
    cast_compute_weights_(m)
    assert m.mlm_out.weight is m.emb.tok.weight and m.mlm_out.weight.dtype == torch.bfloat16
    assert m.emb_ln.weight.dtype == torch.float32
    opt = FusedAdamW(m.parameters(), lr=1e-3)
    dts = sorted(str(fg.param_dtype) for fg in opt.flat_groups)
    assert dts == ["torch.bfloat16", "torch.float32"]
    bf = next(fg for fg in opt.flat_groups if fg.param_dtype == torch.bfloat16)
    # fp32 gradients by default, also for the bf16 compute weights
    assert bf.master.dtype == torch.float32 and bf.lowp.dtype == torch.bfloat16 and bf.grad.dtype == torch.float32
    assert bf.mixed and all(p.grad is None for p in bf.params)
    n = sum(p.numel() for p in {id(p): p for p in m.parameters()}.values())
    assert sum(sum(s.numel for s in fg.slots) for fg in opt.flat_groups) == n
    # bf16 gradients are opt-in
    m2 = cast_compute_weights_(BertBase(vocab=100, seq_len=8, d_model=32, heads=2, d_ff=64, layers=1))
    opt2 = FusedAdamW(m2.parameters(), lr=1e-3, grad_dtype=torch.bfloat16)
    bf2 = next(fg for fg in opt2.flat_groups if fg.param_dtype == torch.bfloat16)
    assert bf2.grad.dtype == torch.bfloat16 and not bf2.mixed


def test_mixed_precision_flat_grads_fold_autograd_grads():
    """bf16 weights + fp32 flat gradient: autograd's bf16 .grad is folded into the fp32 slot
    (post-accumulate hook) before the data-parallel readiness hook, and dropped."""
    from vodascheduler_amd.models import cast_compute_weights_
    from vodascheduler_amd.ops.optim import FusedSGD
    from vodascheduler_amd.parallel.ddp import ElasticDDP
    from vodascheduler_amd.utils.flat import grad_of

    torch.manual_seed(0)
    m = cast_compute_weights_(torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4)))
    ref = cast_compute_weights_(torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4)))
    ref.load_state_dict(m.state_dict())
    opt = FusedSGD(m.parameters(), lr=0.1)
    order = []
    ddp = ElasticDDP(m, None, opt)
    real = ddp._on_grad

    def spy(p):
        order.append((id(p), p.grad is None, float(grad_of(p).abs().sum())))
        real(p)

    for p in m.parameters():
        h = p._post_accumulate_grad_hooks
        # replace DDP's readiness hook (registered last) by the spy
        k = list(h)[-1]
        h[k] = spy
    x = torch.randn(8, 16).bfloat16()
    for _ in range(2):  # grads accumulate in fp32 across two backward passes
        m(x).float().sum().backward()
        ref(x).float().sum().backward()
    for p, q in zip(m.parameters(), ref.parameters()):
        assert p.grad is None
        g = grad_of(p)
        assert g.dtype == torch.float32
        torch.testing.assert_close(g, q.grad.float(), atol=3e-2, rtol=2e-2)
    # the readiness hook saw the folded gradient (fold runs first)
    assert order and all(none and s > 0 for _, none, s in order)
    ddp.finalize()
    assert ddp.calibrated


def test_fused_linear_direct_accumulation_matches_autograd():
    from vodascheduler_amd.ops.dense import FusedLinear
    from vodascheduler_amd.ops.optim import FusedSGD

    torch.manual_seed(0)
    ref = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.GELU(), torch.nn.Linear(32, 8))
    fused = torch.nn.Sequential(FusedLinear(16, 32), torch.nn.GELU(), FusedLinear(32, 8))
    fused.load_state_dict(ref.state_dict())
    opt = FusedSGD(fused.parameters(), lr=0.1)  # flat grads -> in-place accumulation path
    ready = []
    for p in fused.parameters():
        p._voda_grad_ready = ready.append
    x = torch.randn(5, 3, 16)
    for _ in range(2):  # accumulates over two backward passes, like autograd
        ref(x).square().sum().backward()
        fused(x).square().sum().backward()
    assert len(ready) == 8
    for pr, pf in zip(ref.parameters(), fused.parameters()):
        torch.testing.assert_close(pf.grad, pr.grad, atol=1e-5, rtol=1e-5)
    opt.zero_grad()
    assert all(float(p.grad.abs().sum()) == 0 for p in fused.parameters())
    # without flat grads: ordinary autograd gradients
    plain = FusedLinear(16, 8)
    plain(x).sum().backward()
    assert plain.weight.grad is not None and plain.bias.grad.shape == (8,)


def test_fused_bn_batches_tracked_and_state_dict():
    from vodascheduler_amd.ops.batchnorm import FusedBatchNorm2d

    m = FusedBatchNorm2d(8)
    for _ in range(3):
        m(torch.randn(2, 8, 3, 3))
    assert int(m.state_dict()["num_batches_tracked"]) == 3
    m2 = FusedBatchNorm2d(8)
    m2.load_state_dict(m.state_dict())
    m2(torch.randn(2, 8, 3, 3))
    assert int(m2.state_dict()["num_batches_tracked"]) == 4


def test_encoder_residual_grad_sink_matches_autograd(monkeypatch):
    """The residual-stream gradient handed to the sublayer's first GEMM (ops/dense.residual_add
    + FusedLinear sink_in) equals autograd's sum, and the hand-off is actually taken."""
    import vodascheduler_amd.models.layers as L
    from vodascheduler_amd.ops import conv1x1 as C

    torch.manual_seed(0)
    m = L.EncoderLayer(64, 4, 128, act="gelu")
    x = torch.randn(2, 10, 64)
    taken = []
    orig = C.GradSink.take
    monkeypatch.setattr(C.GradSink, "take", lambda self: (lambda g: (taken.append(g is not None), g)[1])(orig(self)))

    def run(on):
        monkeypatch.setattr(L, "USE_GRAD_SINK", on)
        xi = x.clone().requires_grad_(True)
        m.zero_grad()
        m(xi).square().sum().backward()
        return xi.grad.clone(), [p.grad.clone() for p in m.parameters()]

    dx0, g0 = run(False)
    assert taken == []
    dx1, g1 = run(True)
    assert taken == [True, True]
    torch.testing.assert_close(dx1, dx0)
    for a, b in zip(g1, g0):
        torch.testing.assert_close(a, b)


@pytest.mark.parametrize("name,kw", [("sgd", dict(lr=0.1, momentum=0.9, weight_decay=1e-4)),
                                     ("adamw", dict(lr=1e-3, weight_decay=0.01)),
                                     ("rmsprop", dict(lr=1e-3, momentum=0.5, centered=True))])
def test_step_range_pieces_equal_whole_step(name, kw):
    """Per-bucket updates (begin_step + step_range over a partition) == one optimizer.step()."""
    from vodascheduler_amd.ops.optim import make_optimizer

    def build():
        torch.manual_seed(0)
        return torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.Tanh(), torch.nn.Linear(64, 8))

    a, b = build(), build()
    oa, ob = make_optimizer(name, a.parameters(), **kw), make_optimizer(name, b.parameters(), **kw)
    x = torch.randn(32, 16)
    for _ in range(3):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            m(x).square().mean().backward()
        oa.step()
        ob.begin_step()
        n = ob.flat_groups[0].numel
        cuts = [0, 64, 1088, n]  # slot-aligned pieces, applied out of order
        for lo, hi in sorted(zip(cuts[:-1], cuts[1:]), key=lambda r: -r[0]):
            ob.step_range(0, lo, hi)
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa, pb)


def test_ddp_overlap_optimizer_is_opt_in_and_cpu_off():
    from vodascheduler_amd.ops.optim import make_optimizer
    from vodascheduler_amd.parallel.ddp import ElasticDDP

    m = torch.nn.Linear(8, 8)
    o = make_optimizer("sgd", m.parameters(), lr=0.1)
    assert not ElasticDDP(m, None, o).overlap_optimizer
    assert not ElasticDDP(m, None, o, overlap_optimizer=True).overlap_optimizer  # CPU: never


def test_conv_sep_bias_matches_conv2d_and_flat_grad():
    from vodascheduler_amd.ops.conv_bias import Conv2dSepBias
    from vodascheduler_amd.ops.optim import make_optimizer
    from vodascheduler_amd.utils.flat import grad_of

    torch.manual_seed(0)
    ref = torch.nn.Conv2d(4, 8, 3, padding=1)
    m = Conv2dSepBias(4, 8, 3, padding=1)
    m.load_state_dict(ref.state_dict())
    x = torch.randn(2, 4, 9, 7)
    torch.testing.assert_close(m(x), ref(x))
    opt = make_optimizer("sgd", m.parameters(), lr=0.0)  # flat grads: the direct column-sum path
    opt.zero_grad()
    (m(x) ** 2).sum().backward()
    (ref(x) ** 2).sum().backward()
    torch.testing.assert_close(grad_of(m.bias), ref.bias.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(grad_of(m.weight), ref.weight.grad, rtol=1e-5, atol=1e-5)


def test_grad_only_ddp_bf16_params_with_stock_optimizer():
    """ElasticDDP in grad-only mode with bf16 parameters and a stock
    torch.optim optimizer -- the gradients must land in p.grad (bf16 flat buffer), so SGD
    actually updates, exactly as without the engine."""
    from vodascheduler_amd.parallel.ddp import ElasticDDP

    torch.manual_seed(0)
    ref = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4)).to(torch.bfloat16)
    m = copy.deepcopy(ref)
    w0 = next(m.parameters()).detach().clone()
    x = torch.randn(8, 16, dtype=torch.bfloat16)
    o_ref = torch.optim.SGD(ref.parameters(), lr=0.1)
    o = torch.optim.SGD(m.parameters(), lr=0.1)
    ddp = ElasticDDP(m, None, o)
    for _ in range(3):
        o_ref.zero_grad()
        ref(x).float().square().mean().backward()
        o_ref.step()
        ddp.zero_grad()
        m(x).float().square().mean().backward()
        ddp.step()
    for a, b in zip(m.parameters(), ref.parameters()):
        assert a.grad is not None and a.grad.dtype == torch.bfloat16
        assert torch.equal(a, b)
    assert not torch.equal(next(m.parameters()), w0)  # the optimizer did update
