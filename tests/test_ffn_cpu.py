"""Epilogue-fused feed-forward block (ops/ffn.py): the CPU reference path of the fused
autograd function equals the autograd composition fc2(gelu_tanh(fc1(x)))."""
import torch
import torch.nn.functional as F

from vodascheduler_amd.ops import ffn


def test_gelu_tanh_grad_ref_matches_autograd():
    h = torch.linspace(-6, 6, 1001, dtype=torch.float64, requires_grad=True)
    F.gelu(h, approximate="tanh").sum().backward()
    torch.testing.assert_close(ffn.gelu_tanh_grad_ref(h.detach()).double(), h.grad, atol=1e-6, rtol=1e-6)


def test_ffn_function_matches_composition_cpu():
    torch.manual_seed(0)
    x = torch.randn(3, 5, 16, dtype=torch.float64, requires_grad=True)
    w1 = torch.randn(32, 16, dtype=torch.float64, requires_grad=True)
    b1 = torch.randn(32, dtype=torch.float64, requires_grad=True)
    w2 = torch.randn(16, 32, dtype=torch.float64, requires_grad=True)
    b2 = torch.randn(16, dtype=torch.float64, requires_grad=True)
    out = ffn._FFNGeluFn.apply(x, w1, b1, w2, b2, None, None)
    g = torch.randn_like(out)
    grads = torch.autograd.grad(out, (x, w1, b1, w2, b2), g)
    ref = F.linear(F.gelu(F.linear(x, w1, b1), approximate="tanh"), w2, b2)
    rgrads = torch.autograd.grad(ref, (x, w1, b1, w2, b2), g)
    torch.testing.assert_close(out, ref)
    for a, b in zip(grads, rgrads):  # bias gradients are summed in fp32 (as in FusedLinear)
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)


def test_ffn_function_skips_handed_over_bias_gradient():
    """A BiasHandoff marked done (the LayerNorm backward summed fc2's bias gradient) makes the
    FFN backward skip that gradient."""
    from vodascheduler_amd.ops.dense import BiasHandoff

    torch.manual_seed(1)
    x = torch.randn(2, 3, 8, dtype=torch.float64, requires_grad=True)
    w1 = torch.randn(16, 8, dtype=torch.float64, requires_grad=True)
    b1 = torch.randn(16, dtype=torch.float64, requires_grad=True)
    w2 = torch.randn(8, 16, dtype=torch.float64, requires_grad=True)
    b2 = torch.randn(8, dtype=torch.float64, requires_grad=True)
    hb = BiasHandoff(b2)
    out = ffn._FFNGeluFn.apply(x, w1, b1, w2, b2, None, hb)
    hb.done = True
    out.sum().backward()
    assert b2.grad is None and b1.grad is not None and not hb.done
