"""Split-K MFMA weight-gradient kernel (csrc/hip/wgrad.hip) against the fp32 PyTorch
reference: shapes off the 128-tile grid, token counts off the 64-token stage, with and
without accumulation / bias, every split count, and through FusedLinear's backward."""
import pytest
import torch

from vodascheduler_amd.ops import wgrad as W


def test_default_splits_cover_the_chip():
    ds = lambda M, N, K: W.default_splits(M, N, K, variant=2)  # noqa: E731
    assert ds(8192, 768, 768) == 12       # 36 tiles -> 432 workgroups
    assert ds(8192, 3072, 768) == 3       # 144 tiles
    assert ds(8192, 2304, 768) == 4
    assert ds(1280, 768, 768) == 5
    assert ds(300, 768, 768) == 1         # few tokens: no split
    assert ds(8192, 4096, 4096) == 1
    # 256 x 256 tiles, one workgroup per CU
    # 256 x 256 tiles, one workgroup per CU: at most one round of 256 workgroups
    assert W.default_splits(8192, 3072, 768, variant=6) == 7     # 36 tiles -> 252
    assert W.default_splits(8192, 768, 768, variant=9) == 28     # 9 tiles -> 252
    assert W.default_splits(8192, 2304, 768, variant=9) == 9     # 27 tiles -> 243


def test_cpu_path_matches_reference():
    dy, x = torch.randn(70, 24), torch.randn(70, 40)
    gw, gb = torch.randn(24, 40), torch.randn(24)
    w_ref, b_ref = W.wgrad_ref(dy, x, gw, gb)
    W.wgrad_accumulate_(dy, x, gw, gb)
    torch.testing.assert_close(gw, w_ref)
    torch.testing.assert_close(gb, b_ref)


def _case(M, N, K, seed=0, dev="cuda"):
    g = torch.Generator(device=dev).manual_seed(seed)
    dy = torch.randn(M, N, device=dev, generator=g).bfloat16()
    # asymmetric operand so a transposed write or swapped fragment map cannot pass
    x = (torch.randn(M, K, device=dev, generator=g) + torch.arange(K, device=dev) / K).bfloat16()
    gw = torch.randn(N, K, device=dev, generator=g).bfloat16()
    gb = torch.randn(N, device=dev, generator=g).bfloat16()
    return dy, x, gw, gb


def _check(dy, x, gw, gb, accumulate, splits, with_bias=True, variant=None):
    w_ref, b_ref = W.wgrad_ref(dy, x, gw, gb if with_bias else None, accumulate)
    gw2, gb2 = gw.clone(), gb.clone()
    W.wgrad_accumulate_(dy, x, gw2, gb2 if with_bias else None, accumulate=accumulate, splits=splits,
                        variant=variant)
    torch.cuda.synchronize()
    M = dy.shape[0]
    tol = dict(rtol=2e-2, atol=2e-2 * max(1.0, (M / 64) ** 0.5))
    torch.testing.assert_close(gw2.float(), w_ref, **tol)
    if with_bias:
        torch.testing.assert_close(gb2.float(), b_ref, **tol)
    else:
        assert torch.equal(gb2, gb)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(64, 128, 128), (200, 136, 72), (1280, 768, 768), (777, 256, 384),
                                   (8192, 768, 3072)])
@pytest.mark.parametrize("splits", [1, 3, 8])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10])
def test_wgrad_kernel_matches_fp32(M, N, K, splits, variant):
    dy, x, gw, gb = _case(M, N, K)
    _check(dy, x, gw, gb, True, splits, variant=variant)


@pytest.mark.gpu
@pytest.mark.parametrize("splits", [1, 4])
@pytest.mark.parametrize("variant", [0, 1, 4, 6, 7, 9, 10])
def test_wgrad_kernel_overwrite_and_no_bias(splits, variant):
    dy, x, gw, gb = _case(512, 192, 320, seed=3)
    _check(dy, x, gw, gb, False, splits, variant=variant)
    _check(dy, x, gw, gb, True, splits, with_bias=False, variant=variant)


@pytest.mark.gpu
def test_wgrad_kernel_identity_operand():
    # dY = I (first N tokens), X arbitrary -> dW = X[:N] exactly (bf16 values, fp32 sums)
    N, K, M = 128, 256, 192
    dy = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
    dy[:N] = torch.eye(N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda").bfloat16()
    gw = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    gb = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
    for s, v in ((1, 0), (3, 0), (1, 1), (3, 1), (2, 2), (3, 3), (1, 4), (3, 4), (2, 5), (1, 6), (3, 6), (2, 7), (3, 8), (1, 9), (3, 9), (1, 10), (3, 10)):
        gw.zero_()
        gb.zero_()
        W.wgrad_accumulate_(dy, x, gw, gb, splits=s, variant=v)
        torch.testing.assert_close(gw, x[:N], rtol=0, atol=0)
        torch.testing.assert_close(gb, torch.ones(N, device="cuda", dtype=torch.bfloat16), rtol=0, atol=0)


@pytest.mark.gpu
def test_wgrad_strided_rows_and_deterministic():
    base_dy = torch.randn(1024, 1024, device="cuda").bfloat16()
    base_x = torch.randn(1024, 512, device="cuda").bfloat16()
    dy, x = base_dy[:, 128:128 + 768], base_x[:, :256]      # row strides 1024 / 512
    gw = torch.zeros(768, 256, device="cuda", dtype=torch.bfloat16)
    assert W.supported(dy, x, gw)
    for v in (2, 6, 9):
        gw.zero_()
        W.wgrad_accumulate_(dy, x, gw, None, splits=4, variant=v)
        first = gw.clone()
        gw.zero_()
        W.wgrad_accumulate_(dy, x, gw, None, splits=4, variant=v)
        assert torch.equal(first, gw)
        torch.testing.assert_close(first.float(), dy.float().t() @ x.float(), rtol=2e-2, atol=0.5)


@pytest.mark.gpu
def test_fused_linear_backward_uses_kernel_and_matches_autograd():
    from vodascheduler_amd.ops import dense
    from vodascheduler_amd.ops.optim import make_optimizer

    torch.manual_seed(0)
    lin = dense.FusedLinear(768, 3072).cuda().bfloat16()
    ref = torch.nn.Linear(768, 3072).cuda()
    ref.load_state_dict({k: v.float() for k, v in lin.state_dict().items()})
    opt = make_optimizer("sgd", lin.parameters(), lr=0.0)  # flat grads -> direct accumulation path
    x = torch.randn(4, 512, 768, device="cuda")
    assert dense.USE_WGRAD_KERNEL
    opt.zero_grad()
    lin(x.bfloat16()).float().square().mean().backward()
    ref(x.bfloat16().float()).square().mean().backward()
    from vodascheduler_amd.utils.flat import grad_of

    for got, want in ((grad_of(lin.weight), ref.weight.grad), (grad_of(lin.bias), ref.bias.grad)):
        rel = (got.float() - want).norm() / want.norm()
        assert rel < 1e-2, rel


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 2, 6, 9])
@pytest.mark.parametrize("splits", [1, 4])
@pytest.mark.parametrize("accumulate", [True, False])
def test_wgrad_kernel_fp32_output(variant, splits, accumulate):
    """fp32 dW / db (the default flat-gradient precision): the fp32 MFMA accumulators are
    rounded once, so the result matches the fp32 reference to summation-order error."""
    M, N, K = 1000, 264, 392
    dy, x, gw, gb = _case(M, N, K, seed=5)
    gw32, gb32 = gw.float(), gb.float()
    w_ref, b_ref = W.wgrad_ref(dy, x, gw32, gb32, accumulate)
    assert W.supported(dy, x, gw32, gb32)
    W.wgrad_accumulate_(dy, x, gw32, gb32, accumulate=accumulate, splits=splits, variant=variant)
    torch.cuda.synchronize()
    torch.testing.assert_close(gw32, w_ref, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(gb32, b_ref, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
def test_fused_linear_fp32_flat_grad_default_and_bf16_opt_in():
    from vodascheduler_amd.ops import dense
    from vodascheduler_amd.ops.optim import make_optimizer
    from vodascheduler_amd.utils.flat import grad_of

    torch.manual_seed(1)
    x = torch.randn(2048, 768, device="cuda").bfloat16()
    for gdt in (None, torch.bfloat16):
        lin = dense.FusedLinear(768, 768).cuda().bfloat16()
        opt = make_optimizer("sgd", lin.parameters(), lr=0.0, grad_dtype=gdt)
        opt.zero_grad()
        lin(x).float().square().mean().backward()
        g = grad_of(lin.weight)
        assert g.dtype == (gdt or torch.float32)
        want = (2.0 / lin(x).numel()) * (lin(x).float().t() @ x.float())
        rel = float((g.float() - want).norm() / want.norm())
        assert rel < (1e-3 if gdt is None else 1e-2), (gdt, rel)
