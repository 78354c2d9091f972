"""Transformer encoder block on GPU with the fused residual paths on and off:
the LayerNorm(x + residual) kernel and the GradSink hand-off of the residual gradient to
the sublayer's first GEMM, under bf16 autocast with a flat-gradient (fp32) optimizer, with
dropout 0 and > 0 -- against the unfused autograd path."""
import copy

import pytest
import torch


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


@pytest.mark.gpu
@pytest.mark.parametrize("dropout", [0.0, 0.1])
def test_encoder_layer_fused_residual_and_sink_match_unfused(dropout, monkeypatch):
    import vodascheduler_amd.models.layers as L
    from vodascheduler_amd.models import cast_compute_weights_
    from vodascheduler_amd.ops import conv1x1
    from vodascheduler_amd.ops.optim import make_optimizer
    from vodascheduler_amd.utils.flat import grad_of

    torch.manual_seed(0)
    base = L.EncoderLayer(256, 4, 1024, act="gelu", dropout=dropout).cuda()
    x0 = torch.randn(8, 64, 256, device="cuda")
    mask = torch.ones(8, 64, dtype=torch.bool, device="cuda")
    mask[:, -5:] = False
    puts = []
    real_put = conv1x1.GradSink.put

    def counting_put(self, g):
        puts.append(g.shape)
        real_put(self, g)

    monkeypatch.setattr(conv1x1.GradSink, "put", counting_put)

    def run(fused, sink):
        monkeypatch.setattr(L, "FUSED_RESIDUAL_LN", fused)
        monkeypatch.setattr(L, "USE_GRAD_SINK", sink)
        m = cast_compute_weights_(copy.deepcopy(base)).train()
        opt = make_optimizer("sgd", m.parameters(), lr=0.0)
        opt.zero_grad()
        x = x0.bfloat16().requires_grad_(True)
        torch.manual_seed(123)  # same dropout masks in every configuration
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            y = m(x, key_mask=mask)
        y.float().square().mean().backward()
        torch.cuda.synchronize()
        return x.grad.float(), {n: grad_of(p).float().clone() for n, p in m.named_parameters()}

    dx_ref, pg_ref = run(False, False)
    assert not puts
    for fused, sink in ((True, False), (False, True), (True, True)):
        n0 = len(puts)
        dx, pg = run(fused, sink)
        if sink:
            assert len(puts) - n0 == 2, "the residual-gradient hand-off was not taken"
        assert _rel(dx, dx_ref) < 2e-2, (fused, sink, _rel(dx, dx_ref))
        for n in pg_ref:
            assert _rel(pg[n], pg_ref[n]) < 3e-2, (fused, sink, n, _rel(pg[n], pg_ref[n]))


@pytest.mark.gpu
def test_fp32_encoder_bias_handoffs_match_unfused(monkeypatch):
    """fp32 BERT-style encoder layer with flat gradients: the two sublayers' output-projection
    bias gradients from the LayerNorm backwards (ops/dense.BiasHandoff) equal the Linear column
    sums of the unfused path; those two Linears skip their own column-sum pass."""
    import vodascheduler_amd.models.layers as L
    from vodascheduler_amd.ops import dense
    from vodascheduler_amd.ops.optim import make_optimizer
    from vodascheduler_amd.utils.flat import grad_of

    torch.manual_seed(0)
    base = L.EncoderLayer(256, 4, 1024, act="gelu", dropout=0.0).cuda()
    x0 = torch.randn(8, 64, 256, device="cuda")
    seen = []
    real = dense.linear_weight_grads

    def spy(dy2, x2, weight, bias, need_w, need_b):
        seen.append(need_b)
        return real(dy2, x2, weight, bias, need_w, need_b)

    monkeypatch.setattr(dense, "linear_weight_grads", spy)

    real_target = dense.BiasHandoff.target

    def run(fused):
        # reference: every handoff declines (the Linears sum their own bias gradients)
        monkeypatch.setattr(dense.BiasHandoff, "target", real_target if fused else (lambda self, dtype: None))
        m = copy.deepcopy(base).train()
        opt = make_optimizer("sgd", m.parameters(), lr=0.0)
        opt.zero_grad()
        x = x0.clone().requires_grad_(True)
        m(x).square().mean().backward()
        torch.cuda.synchronize()
        return x.grad, {n: grad_of(p).clone() for n, p in m.named_parameters()}

    dx_ref, pg_ref = run(False)
    assert all(seen) and len(seen) == 4
    seen.clear()
    dx, pg = run(True)
    assert sorted(seen) == [False, False, True, True], seen  # qkv and fc1 sum their own biases
    assert _rel(dx, dx_ref) < 1e-5
    for n in pg_ref:
        assert _rel(pg[n], pg_ref[n]) < 1e-5, (n, _rel(pg[n], pg_ref[n]))
