"""hipBLASLt GEMMs with the GELU epilogues (csrc/hip/blaslt_epi.cpp, ops/ffn.py) against fp32
PyTorch references, and the epilogue-fused FeedForward / EncoderLayer against the unfused
FusedLinear -> GELU kernel -> FusedLinear path."""
import pytest
import torch
import torch.nn.functional as F

from vodascheduler_amd.ops import ffn

pytestmark = pytest.mark.gpu


def test_epilogue_probe_runs():
    """The capability probe answers (>= 0 algorithms) for every epilogue the FFN may use;
    plain GELU_BIAS always has kernels."""
    from vodascheduler_amd.ops import _native

    h = _native.hip()
    assert h.gemm_epilogue_algos(36, True, 3072, 8192, 768) > 0
    for e in (ffn.EPI_GELU_AUX_BIAS, ffn.EPI_DGELU):
        assert h.gemm_epilogue_algos(e, False, 3072, 8192, 768) >= 0
    ffn.epilogues_available(torch.device("cuda", 0))


needs_epi = pytest.mark.skipif(
    not (torch.cuda.is_available() and ffn.epilogues_available(torch.device("cuda", 0))),
    reason="this hipBLASLt has no GELU_AUX_BIAS / DGELU kernels (gfx950, ROCm 7.x)")


@needs_epi
@pytest.mark.parametrize("M,N,K", [(8192, 3072, 768), (256, 64, 32), (1000, 136, 48)])
def test_gemm_gelu_aux_matches_fp32(M, N, K):
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    h, y = ffn.gemm_gelu_aux(x, w, b)
    hr = x.float() @ w.float().t() + b.float()
    torch.testing.assert_close(h.float(), hr, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(y.float(), F.gelu(hr, approximate="tanh"), atol=3e-2, rtol=2e-2)


@needs_epi
@pytest.mark.parametrize("M,N,K", [(8192, 768, 3072), (256, 32, 64), (1000, 48, 136)])
def test_gemm_dgelu_matches_fp32(M, N, K):
    torch.manual_seed(1)
    dy = torch.randn(M, N, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / N ** 0.5).bfloat16()
    h = (torch.randn(M, K, device="cuda") * 2).bfloat16()
    dh = ffn.gemm_dgelu(dy, w, h)
    ref = (dy.float() @ w.float()) * ffn.gelu_tanh_grad_ref(h.float())
    torch.testing.assert_close(dh.float(), ref, atol=3e-2, rtol=2e-2)


@needs_epi
@pytest.mark.parametrize("sink", [False, True])
def test_encoder_layer_epilogue_ffn_matches_unfused(sink, monkeypatch):
    from vodascheduler_amd.models import layers as L

    torch.manual_seed(0)
    layer = L.EncoderLayer(128, 4, 512, act="gelu").cuda()
    for p in layer.parameters():
        if p.dim() == 2:
            p.data = p.data.bfloat16()
    for m in layer.modules():
        if isinstance(m, torch.nn.Linear) and m.bias is not None:
            m.bias.data = m.bias.data.bfloat16()
    x0 = torch.randn(4, 32, 128, device="cuda").bfloat16()
    g = torch.randn(4, 32, 128, device="cuda").bfloat16()
    monkeypatch.setattr(L, "USE_GRAD_SINK", sink)

    def run(epi):
        monkeypatch.setattr(ffn, "USE_GELU_EPILOGUE", epi)
        layer.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            y = layer(x)
        y.backward(g)
        return [y.float(), x.grad.float()] + [p.grad.float() for p in layer.parameters()]

    fused, plain = run(True), run(False)
    for i, (a, b) in enumerate(zip(fused, plain)):
        scale = b.abs().max().item() + 1e-6
        assert (a - b).abs().max().item() <= 3e-2 * scale + 1e-2, f"tensor {i}"
