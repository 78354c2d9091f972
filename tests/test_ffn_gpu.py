"""hipBLASLt GEMMs with the GELU epilogues (csrc/hip/blaslt_epi.cpp, ops/ffn.py) against fp64
PyTorch references, and the epilogue-fused FeedForward / EncoderLayer against the unfused
FusedLinear -> GELU kernel -> FusedLinear path (fp32, the reference's precision)."""
import pytest
import torch
import torch.nn.functional as F

from vodascheduler_amd.ops import ffn

pytestmark = pytest.mark.gpu


def test_epilogue_probe_runs():
    """The capability probe answers for both dtypes; plain GELU_BIAS always has kernels, and on
    gfx950 / ROCm 7.2 fp32 has both FFN epilogues (the path BERT fp32 takes)."""
    from vodascheduler_amd.ops import _native

    h = _native.hip()
    assert h.gemm_epilogue_algos(36, 0, True, 3072, 8192, 768) > 0
    for dt in (0, 1):
        for e in (ffn.EPI_GELU_AUX_BIAS, ffn.EPI_DGELU):
            assert h.gemm_epilogue_algos(e, dt, False, 3072, 8192, 768) >= 0
    assert ffn.epilogues_available(torch.device("cuda", 0), torch.float32)
    ffn.epilogues_available(torch.device("cuda", 0), torch.bfloat16)
    # the per-shape check covers the backward's DGELU GEMM of the real token count
    assert ffn.shape_available(torch.device("cuda", 0), torch.float32, 8192, 768, 3072)
    assert isinstance(ffn.shape_available(torch.device("cuda", 0), torch.float32, 24, 768, 3072), bool)


@pytest.mark.parametrize("M,N,K", [(8192, 3072, 768), (256, 64, 32), (1000, 136, 48)])
def test_gemm_gelu_aux_matches_fp64(M, N, K):
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda")
    h, y = ffn.gemm_gelu_aux(x, w, b)
    hr = x.double() @ w.double().t() + b.double()
    torch.testing.assert_close(h.double(), hr, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(y.double(), F.gelu(hr, approximate="tanh"), atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("M,N,K", [(8192, 768, 3072), (256, 32, 64), (1000, 48, 136)])
def test_gemm_dgelu_matches_fp64(M, N, K):
    torch.manual_seed(1)
    dy = torch.randn(M, N, device="cuda")
    w = torch.randn(N, K, device="cuda") / N ** 0.5
    h = torch.randn(M, K, device="cuda") * 2
    dh = ffn.gemm_dgelu(dy, w, h)
    ref = (dy.double() @ w.double()) * ffn.gelu_tanh_grad_ref(h.double())
    torch.testing.assert_close(dh.double(), ref, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("sink", [False, True])
def test_fp32_encoder_layer_epilogue_ffn_matches_unfused(sink, monkeypatch):
    """fp32 EncoderLayer (GELU FFN, bias hand-offs on) with the epilogue FFN vs the unfused FFN:
    outputs and every gradient agree to fp32 rounding; the fused path really ran."""
    from vodascheduler_amd.models import layers as L

    torch.manual_seed(0)
    layer = L.EncoderLayer(128, 4, 512, act="gelu").cuda()
    x0 = torch.randn(4, 32, 128, device="cuda")
    g = torch.randn(4, 32, 128, device="cuda")
    monkeypatch.setattr(L, "USE_GRAD_SINK", sink)
    calls = []
    real = ffn._FFNGeluFn.apply

    def spy(*a):
        calls.append(1)
        return real(*a)

    monkeypatch.setattr(ffn._FFNGeluFn, "apply", spy)

    def run(epi):
        monkeypatch.setattr(ffn, "USE_GELU_EPILOGUE", epi)
        layer.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_()
        y = layer(x)
        y.backward(g)
        return [y, x.grad] + [p.grad for p in layer.parameters()]

    fused = run(True)
    assert calls == [1]
    plain = run(False)
    assert calls == [1]
    for i, (a, b) in enumerate(zip(fused, plain)):
        rel = ((a.double() - b.double()).norm() / (b.double().norm() + 1e-12)).item()
        assert rel < 1e-5, f"tensor {i}: {rel}"
