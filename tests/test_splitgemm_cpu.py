"""CPU numerics of the exact 3-way bf16 split behind csrc/hip/splitgemm.hip: the split is
exact, and the six kept cross products reproduce an fp32-accurate product (host model with
the bf16 products emulated in fp64) -- the algorithm the GPU kernel runs."""
import torch

from vodascheduler_amd.ops import splitgemm as SG


def test_split3_is_exact():
    torch.manual_seed(0)
    x = torch.randn(4096) * torch.exp2(torch.randint(-60, 61, (4096,)).float())
    hi, mid, lo = SG.split3(x)
    for t in (hi, mid, lo):  # every part is a bf16 value
        assert torch.equal(t, t.to(torch.bfloat16).float())
    assert torch.equal(hi.double() + mid.double() + lo.double(), x.double())
    # magnitudes: mid <= 2^-8 |hi|, lo <= 2^-16 |hi| (round-to-nearest halves them)
    nz = hi != 0
    assert (mid[nz].abs() <= hi[nz].abs() * 2.0 ** -8).all()
    assert (lo[nz].abs() <= hi[nz].abs() * 2.0 ** -16).all()


def _err(c, a, b):
    ref = a.double() @ b.double()
    return ((c.double() - ref).abs() / (a.double().abs() @ b.double().abs())).max().item()


def test_six_products_fp32_accurate():
    torch.manual_seed(1)
    a = torch.randn(64, 2048)
    b = torch.randn(2048, 64)
    e6 = _err(SG.emulate(a, b, 6), a, b)
    e9 = _err(SG.emulate(a, b, 9), a, b)
    e3 = _err(SG.emulate(a, b, 3), a, b)
    # dropped terms <= ~3 * 2^-24 per product with random signs: far below fp32 rounding
    assert e6 < 2.0 ** -24 / 16, e6
    assert e9 < 1e-12, e9              # the full expansion is exact up to fp64 accumulation
    assert e3 > 100 * e6, (e3, e6)     # a 2-way split is ~16-bit: not fp32-accurate
    # and no worse than a plain fp32 GEMM's rounding on the same data
    assert e6 <= 1.5 * _err(a @ b, a, b) + 2.0 ** -24


def test_wide_magnitudes():
    torch.manual_seed(2)
    a = torch.randn(32, 512) * torch.exp2(torch.randint(-30, 31, (32, 512)).float())
    b = torch.randn(512, 32) * torch.exp2(torch.randint(-30, 31, (512, 32)).float())
    assert _err(SG.emulate(a, b, 6), a, b) < 2.0 ** -24 * 3


def test_cpu_matmul_reference_and_layouts():
    torch.manual_seed(3)
    x = torch.randn(24, 32)
    w = torch.randn(16, 32)
    bias = torch.randn(16)
    y = SG.linear(x, w, bias)
    assert torch.allclose(y, x @ w.t() + bias, atol=1e-5)
    # layout detection: K-contiguous / K-major for both operands
    assert SG._layout(x, True) == (False, 32)
    assert SG._layout(x.t().contiguous().t(), True) == (True, 24)
    assert SG._layout(w.t(), False) == (False, 32)
    assert SG._layout(w, False) == (True, 32)
    assert not SG.supported(x, w.t())  # CPU tensors never take the GPU kernel
