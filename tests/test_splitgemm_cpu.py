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


def test_choose_tiles_and_splits():
    """The launch-shape rules from the round-6 sweeps (profiles/r6/splitgemm_t7_sweep.jsonl,
    splitgemm_wgrad_splits.jsonl): 128 x 96 where it fills whole rounds of the 512 resident
    workgroups, 7 / 12 splits for the BERT-base weight gradients, 128 x 128 elsewhere."""
    assert SG.choose(8192, 2304, 768) == (7, 1)     # qkv forward: 1536 tiles of 128 x 96
    assert SG.choose(8192, 768, 768) == (7, 1)      # o forward / input gradient: 512 tiles
    assert SG.choose(8192, 768, 2304) == (7, 1)     # qkv input gradient
    assert SG.choose(8192, 3072, 768) == (0, 1)     # fc1 forward: 1536 tiles of 128 x 128 already
    assert SG.choose(8192, 768, 3072) == (0, 2)     # long K: 128 x 128 with split-K 2
    assert SG.choose(768, 2304, 8192) == (0, 7)     # weight gradients
    assert SG.choose(3072, 768, 8192) == (0, 7)
    assert SG.choose(768, 768, 8192) == (0, 12)
    old = SG.USE_T7
    try:
        SG.USE_T7 = False
        assert SG.choose(8192, 2304, 768) == (0, 1)
    finally:
        SG.USE_T7 = old


def test_plan_variant_8_for_kmajor_b():
    """Input / weight gradients (K-major B) and forwards plan variant 8 on 128 x 128 tiles with
    the same split-K rules, except where a whole 128 x 96 round wins; pinned tiles keep the default (profiles/r6/splitgemm_v8_3wg_probe.jsonl)."""
    x = torch.zeros(64, 32)
    w = torch.zeros(32, 48)  # B [K, N] row-major: K-major (dX = dY W, dW = dY^T X)
    assert SG.plan_variant(True) == (8 if SG.USE_V8_KMAJOR_B else 0)
    assert SG.plan_variant(True, tile=7) == SG.DEFAULT_VARIANT
    assert SG.plan_variant(False) == (8 if SG.USE_V8_FWD else 0)
    assert SG.plan(x, w)[2] == SG.plan_variant(True)
    assert SG.plan(x, w.t().contiguous().t())[2] == SG.plan_variant(False)
    if SG.USE_V8_KMAJOR_B and SG.USE_V8_FWD and SG.USE_T7:
        assert SG.plan_variant(True, None, 8192, 768, 768) == 0     # o input gradient: a t7 round
        assert SG.plan_variant(False, None, 8192, 768, 768) == 0    # o forward
        assert SG.plan_variant(True, None, 8192, 768, 2304) == 8    # qkv input gradient (split-K 2)
        assert SG.plan_variant(False, None, 8192, 2304, 768) == 8   # qkv forward: 1152 tiles
        assert SG.plan_variant(False, None, 8192, 3072, 768) == 8   # fc1 forward
    assert SG.choose(8192, 768, 2304, 8) == (0, 2)     # qkv input gradient: 384 tiles, no 128 x 96
    assert SG.choose(8192, 2304, 768, 8) == ((7, 1) if SG.USE_T7_V8 else (0, 1))  # qkv forward: 2 rounds
    assert SG.choose(8192, 3072, 768, 8) == (0, 1)     # fc1 forward: 1536 tiles fill 2 rounds already
    assert SG.choose(8192, 768, 3072, 8) == (0, 2)
    assert SG.choose(768, 2304, 8192, 8) == (0, 7)
    assert SG.choose(768, 768, 8192, 8) == (0, 12)
    rs = torch.zeros(64)
    assert not SG.row_sums_ok(x.t(), rs, 7, 8)        # CPU tensors never fuse anyway
    old = SG.USE_V8_KMAJOR_B
    try:
        SG.USE_V8_KMAJOR_B = False
        assert SG.plan_variant(True) == SG.DEFAULT_VARIANT
        assert SG.plan_variant(False) == (8 if SG.USE_V8_FWD else 0)
    finally:
        SG.USE_V8_KMAJOR_B = old


def test_thin_tiles_and_wgrad_splits():
    assert SG.thin_tile(64, 256) == 5 and SG.thin_tile(256, 64) == 6 and SG.thin_tile(128, 256) == 0
    # ~target workgroups, >= 256 pixels per split
    assert SG.conv_wgrad_splits(64, 256, 802816, 5, 512) == 512
    assert SG.conv_wgrad_splits(512, 128, 200704, 0, 512) == 128
    assert SG.conv_wgrad_splits(128, 1152, 200704) == 113      # 3x3: ~1024 workgroups
    assert SG.conv_wgrad_splits(2048, 512, 12544, 0, 512) == 8


def test_conv_cpu_references():
    """CPU tensors take the PyTorch reference of the implicit-GEMM convolutions."""
    torch.manual_seed(2)
    x = torch.randn(2, 16, 9, 9)
    w = torch.randn(8, 16, 3, 3)
    torch.testing.assert_close(SG.conv_fwd(x, w, 2, 1), torch.nn.functional.conv2d(x, w, None, 2, 1))
    dy = torch.randn(2, 8, 5, 5)
    ref = torch.nn.grad.conv2d_input((2, 16, 9, 9), w, dy, stride=2, padding=1)
    torch.testing.assert_close(SG.conv_dgrad_s2(dy, w, (2, 16, 9, 9)), ref)


def test_polyphase_taps_cover_the_stride2_input_gradient():
    """Host model of conv_dgrad_s2's decomposition: the four parity classes with their 1 / 2 / 2
    / 4 taps (kh = 1 for even rows; kh = 2, 0 at dY rows i, i + 1 for odd rows) reproduce the
    stride-2 pad-1 input gradient exactly in fp64."""
    torch.manual_seed(3)
    n, cin, cout, H = 2, 4, 3, 9
    w = torch.randn(cout, cin, 3, 3, dtype=torch.float64)
    ho = (H - 1) // 2 + 1
    dy = torch.randn(n, cout, ho, ho, dtype=torch.float64)
    ref = torch.nn.grad.conv2d_input((n, cin, H, H), w, dy, stride=2, padding=1)
    dx = torch.zeros_like(ref)
    dyp = torch.nn.functional.pad(dy, (0, 1, 0, 1))  # zero past the map
    for ph in (0, 1):
        for pw in (0, 1):
            hc, wc = (H - ph + 1) // 2, (H - pw + 1) // 2
            acc = torch.zeros(n, cin, hc, wc, dtype=torch.float64)
            for th, kh in enumerate(SG._S2_TAPS[ph]):
                for tw, kw in enumerate(SG._S2_TAPS[pw]):
                    g = dyp[:, :, th:th + hc, tw:tw + wc]
                    acc += torch.einsum("nohw,oi->nihw", g, w[:, :, kh, kw])
            dx[:, :, ph::2, pw::2] = acc
    torch.testing.assert_close(dx, ref)
