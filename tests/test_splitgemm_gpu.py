"""GPU numerics of the split-bf16 fp32 GEMM (csrc/hip/splitgemm.hip) against fp64 references:
all four operand orientations, ragged M / N tiles, split-K, the three tiles, the bias /
accumulate / GELU / DGELU epilogues, and an error bound no worse than hipBLASLt fp32's."""
import pytest
import torch

from vodascheduler_amd.ops import splitgemm as SG
from vodascheduler_amd.ops.ffn import gelu_tanh_grad_ref

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _orient(a, b, akm, bkm):
    """Views of the same a [M, K] / b [K, N] values in the requested memory orientation."""
    a_v = a.t().contiguous().t() if akm else a.contiguous()
    b_v = b.contiguous() if bkm else b.t().contiguous().t()
    return a_v, b_v


def _bound(a, b):
    return a.double().abs() @ b.double().abs()


@pytest.mark.parametrize("akm", [False, True])
@pytest.mark.parametrize("bkm", [False, True])
@pytest.mark.parametrize("tile", [0, 1, 2, 7])
def test_orientations_ragged(akm, bkm, tile):
    torch.manual_seed(tile * 4 + 2 * akm + bkm)
    M, K, N = 388, 272, 196  # ragged in M and N for every tile
    a = torch.randn(M, K, device=DEV)
    b = torch.randn(K, N, device=DEV)
    av, bv = _orient(a, b, akm, bkm)
    assert SG.supported(av, bv)
    c = SG.matmul(av, bv, tile=tile, splits=1)
    ref = a.double() @ b.double()
    err = ((c.double() - ref).abs() / _bound(a, b)).max().item()
    assert err < 2e-7, err


@pytest.mark.parametrize("akm", [False, True])
@pytest.mark.parametrize("bkm", [False, True])
@pytest.mark.parametrize("variant", [6, 7, 8])
def test_wave_specialised_orientations_ragged(akm, bkm, variant):
    """The wave-specialised kernel (4 MFMA + 4 staging waves) on every orientation, ragged tiles,
    odd and even stage counts."""
    torch.manual_seed(2 * akm + bkm + variant)
    for M, K, N in ((388, 272, 196), (132, 16, 260), (256, 48, 128)):
        a = torch.randn(M, K, device=DEV)
        b = torch.randn(K, N, device=DEV)
        av, bv = _orient(a, b, akm, bkm)
        c = SG.matmul(av, bv, tile=0, splits=1, variant=variant)
        ref = a.double() @ b.double()
        err = ((c.double() - ref).abs() / _bound(a, b)).max().item()
        assert err < (2e-7 if variant == 6 else 4e-7), (M, K, N, err)  # 7 / 8: one accumulator


@pytest.mark.parametrize("tile", [5, 6])
@pytest.mark.parametrize("akm", [False, True])
@pytest.mark.parametrize("bkm", [False, True])
def test_thin_tiles(tile, akm, bkm):
    """64 x 256 / 256 x 64 tiles (the 128-byte-row K-major image), every orientation, ragged and
    exact outputs, split-K into an accumulated C."""
    torch.manual_seed(tile + 2 * akm + bkm)
    for M, K, N, s in ((64, 512, 256, 1), (64, 1024, 516, 4), (256, 512, 64, 1), (516, 1024, 64, 4),
                       (100, 272, 196, 1)):
        a = torch.randn(M, K, device=DEV)
        b = torch.randn(K, N, device=DEV)
        av, bv = _orient(a, b, akm, bkm)
        c0 = torch.randn(M, N, device=DEV)
        c = c0.clone()
        SG.matmul(av, bv, out=c, accumulate=True, tile=tile, splits=s)
        ref = a.double() @ b.double() + c0.double()
        err = ((c.double() - ref).abs() / (_bound(a, b) + 1)).max().item()
        assert err < 2e-7, (tile, M, K, N, err)


@pytest.mark.parametrize("splits,variant", [(2, 0), (3, 0), (7, 0), (3, 6), (7, 6), (2, 8), (7, 8)])
def test_split_k_matches_reference(splits, variant):
    torch.manual_seed(splits)
    M, K, N = 256, 1024, 384
    a = torch.randn(K, M, device=DEV).t()  # K-major a, as in a weight gradient
    b = torch.randn(K, N, device=DEV)
    c = SG.matmul(a, b, tile=0, splits=splits, variant=variant)
    ref = a.double() @ b.double()
    assert ((c.double() - ref).abs() / _bound(a, b)).max().item() < (4e-7 if variant == 8 else 2e-7)


@pytest.mark.parametrize("groups", [-1, 1, 2, 4, 16])
def test_split_k_reduce_slab_groups(groups, monkeypatch):
    """The split-K reduce with 1-16 slab groups per column (LDS combine) on a small output with
    many slabs (the ResNet 1x1 weight-gradient shape class), accumulating into C."""
    monkeypatch.setattr(SG, "REDUCE_GROUPS", groups)
    torch.manual_seed(groups + 3)
    M, K, N = 64, 16 * 200, 260
    a = torch.randn(K, M, device=DEV).t()
    b = torch.randn(K, N, device=DEV)
    c0 = torch.randn(M, N, device=DEV)
    c = c0.clone()
    SG.matmul(a, b, out=c, accumulate=True, tile=0, splits=100)
    ref = a.double() @ b.double() + c0.double()
    assert ((c.double() - ref).abs() / (_bound(a, b) + 1)).max().item() < 2e-7
    monkeypatch.setattr(SG, "REDUCE_GROUPS", -1)
    SG.matmul(a, b, out=c, tile=0, splits=2)  # back to the automatic setting


def test_no_worse_than_hipblaslt_wide_magnitudes():
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.manual_seed(5)
    M, K, N = 512, 768, 512
    a = torch.randn(M, K, device=DEV) * torch.exp2(torch.randint(-30, 31, (M, K), device=DEV).float())
    b = torch.randn(K, N, device=DEV) * torch.exp2(torch.randint(-30, 31, (K, N), device=DEV).float())
    ref = a.double() @ b.double()
    bd = _bound(a, b)
    e_lib = ((torch.mm(a, b).double() - ref).abs() / bd).max().item()
    e_sx = ((SG.matmul(a, b).double() - ref).abs() / bd).max().item()
    assert e_sx <= 1.5 * e_lib, (e_sx, e_lib)


@pytest.mark.parametrize("tile", [None, 7])
def test_epilogues_bias_accumulate_gelu_dgelu(tile, monkeypatch):
    """Epilogues on the planned launch (variant 8) and on tile 7 (variant 8 where planned, the
    dual form for the pinned-variant calls)."""
    if tile is not None:  # route every call of this test to the given tile
        monkeypatch.setattr(SG, "choose", lambda M, N, K, variant=0: (tile, 1))
    torch.manual_seed(9)
    M, K, N = 320, 160, 192
    x = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV) * 0.1
    bias = torch.randn(N, device=DEV)
    ref = x.double() @ w.double().t()
    bd = _bound(x, w.t())
    # bias
    tol = 4e-7 if SG.plan(x, w.t())[2] == 8 else 2e-7  # 8: one accumulator
    y = SG.matmul(x, w.t(), bias=bias)
    assert ((y.double() - ref - bias.double()).abs() / (bd + 1)).max().item() < tol
    # accumulate into an existing output (beta = 1), split-K path too
    for s in (1, 4):
        acc = torch.randn(M, N, device=DEV)
        want = acc.double() + ref
        SG.matmul(x, w.t(), out=acc, accumulate=True, splits=s)
        assert ((acc.double() - want).abs() / (bd + 1)).max().item() < tol
    # GELU: aux = h = xW^T + b, out = gelu(h)
    h = torch.empty(M, N, device=DEV)
    g = SG.matmul(x, w.t(), bias=bias, epi=SG.EPI_GELU, aux=h)
    href = ref + bias.double()
    assert ((h.double() - href).abs() / (bd + 1)).max().item() < tol
    gref = torch.nn.functional.gelu(href, approximate="tanh")
    assert (g.double() - gref).abs().max().item() < 1e-5
    # DGELU: out = (dY W) * gelu'(h), h [M, K]
    dy = torch.randn(M, N, device=DEV)
    hh = torch.randn(M, K, device=DEV)
    d = SG.matmul(dy, w, epi=SG.EPI_DGELU, aux=hh)
    dref = (dy.double() @ w.double()) * gelu_tanh_grad_ref(hh.double())
    assert ((d.double() - dref).abs() / (_bound(dy, w) + 1)).max().item() < 1e-5


@pytest.mark.parametrize("akm", [False, True])
@pytest.mark.parametrize("bkm", [False, True])
def test_tile7_variant8_orientations_epilogue(akm, bkm):
    """Variant 8 on 128 x 96 tiles (one accumulator, three workgroups per CU): every operand
    orientation, ragged M / N, bias + GELU epilogue, against fp64."""
    torch.manual_seed(11 + 2 * akm + bkm)
    M, K, N = 324, 208, 196
    a = torch.randn(M, K, device=DEV)
    b = torch.randn(K, N, device=DEV) * 0.1
    av = a.t().contiguous().t() if akm else a
    bv = b if bkm else b.t().contiguous().t()
    bias = torch.randn(N, device=DEV)
    h = torch.empty(M, N, device=DEV)
    g = SG.matmul(av, bv, bias=bias, epi=SG.EPI_GELU, aux=h, tile=7, splits=1, variant=8)
    ref = a.double() @ b.double() + bias.double()
    assert ((h.double() - ref).abs() / (_bound(a, b) + 1)).max().item() < 4e-7
    gref = torch.nn.functional.gelu(ref, approximate="tanh")
    assert (g.double() - gref).abs().max().item() < 1e-5


def test_variants_error_ordering():
    """9 products <= 6 products (dual) ~ hipBLASLt << 3 products (16-bit)."""
    torch.manual_seed(3)
    a = torch.randn(256, 1024, device=DEV)
    b = torch.randn(1024, 256, device=DEV)
    ref = a.double() @ b.double()
    bd = _bound(a, b)
    e = {v: ((SG.matmul(a, b, tile=0, splits=1, variant=v).double() - ref).abs() / bd).max().item()
         for v in SG.VARIANT_NAMES}
    assert e[0] < 2e-7 and e[2] < 2e-7 and e[1] < 4e-7
    assert e[3] > 10 * e[0]


@pytest.mark.parametrize("n,cin,cout,hw,stride", [(2, 128, 128, 16, 1), (3, 64, 132, 8, 1), (16, 128, 128, 7, 1),
                                                  (2, 128, 256, 16, 2), (4, 256, 128, 7, 2), (2, 64, 64, 16, 1),
                                                  (4, 128, 64, 8, 1), (3, 64, 64, 7, 2)])
@pytest.mark.parametrize("ws", [0, 1, 3])
def test_conv_wgrad_implicit_gemm_matches_fp64(n, cin, cout, hw, stride, ws, monkeypatch):
    """dW (+)= conv weight gradient of a 3x3 pad-1 convolution (NHWC gather per tap in the
    B-operand staging, zero padding, stride 1 / 2, ragged maps) against fp64; one-role (dual
    accumulators), wave-specialised and one-role single-accumulator three-workgroup kernels."""
    torch.manual_seed(cin + cout + hw + stride)
    monkeypatch.setattr(SG, "CONV_WGRAD_WS", 1 if ws == 1 else 0)
    monkeypatch.setattr(SG, "CONV_WGRAD_V8", ws == 3)
    cl = torch.channels_last
    x = torch.randn(n, cin, hw, hw, device=DEV).contiguous(memory_format=cl)
    ho = (hw + 2 - 3) // stride + 1
    if (n * ho * ho) % 16:
        pytest.skip("pixel count not a multiple of 16")
    dy = torch.randn(n, cout, ho, ho, device=DEV).contiguous(memory_format=cl)
    gw = torch.randn(cout, cin, 3, 3, device=DEV).contiguous(memory_format=cl)
    g0 = gw.clone()
    assert SG.conv_wgrad_ok(dy, x, gw)
    SG.conv_wgrad_(dy, x, gw, stride, 1, accumulate=True)
    ref = torch.nn.grad.conv2d_weight(x.double(), gw.shape, dy.double(), stride=stride, padding=1)
    bound = torch.nn.grad.conv2d_weight(x.double().abs(), gw.shape, dy.double().abs(), stride=stride, padding=1)
    err = ((gw.double() - g0.double() - ref).abs() / (bound + 1)).max().item()
    assert err < 1e-6, err


@pytest.mark.parametrize("n,cin,cout,hw,stride,k", [(2, 128, 128, 56, 2, 3), (3, 256, 256, 28, 2, 3), (2, 512, 512, 14, 2, 3),
                                                    (3, 64, 132, 9, 1, 3), (2, 32, 64, 7, 2, 1), (1, 16, 8, 5, 1, 3)])
@pytest.mark.parametrize("v8", [False, True])
def test_conv_fwd_implicit_gemm_matches_fp64(n, cin, cout, hw, stride, k, v8, monkeypatch):
    """y = conv2d(x, w, stride, pad) as one implicit GEMM (NHWC gather per tap in the A staging,
    zero padding, stride 1 / 2, ragged pixel counts) against fp64; dual-accumulator and
    single-accumulator three-workgroup images."""
    monkeypatch.setattr(SG, "CONV_FWD_V8", v8)
    torch.manual_seed(cin + cout + hw + stride)
    cl = torch.channels_last
    pad = k // 2
    x = torch.randn(n, cin, hw, hw, device=DEV).contiguous(memory_format=cl)
    w = (torch.randn(cout, cin, k, k, device=DEV) / (k * cin ** 0.5)).contiguous(memory_format=cl)
    assert SG.conv_fwd_ok(x, w)
    y = SG.conv_fwd(x, w, stride, pad)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), None, stride, pad)
    bound = torch.nn.functional.conv2d(x.double().abs(), w.double().abs(), None, stride, pad)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=cl)
    err = ((y.double() - ref).abs() / (bound + 1e-30)).max().item()
    assert err < (4e-7 if v8 else 2e-7), err


@pytest.mark.parametrize("n,cin,cout,hw", [(2, 128, 128, 56), (2, 256, 256, 28), (3, 512, 512, 14), (3, 64, 48, 7),
                                           (2, 32, 16, 9), (1, 16, 32, 8)])
@pytest.mark.parametrize("v8", [False, True])
def test_conv_dgrad_stride2_polyphase_matches_fp64(n, cin, cout, hw, v8, monkeypatch):
    """dX of a stride-2 pad-1 3x3 convolution as four parity-class implicit GEMMs (odd and even
    input sizes) against fp64; dual- and single-accumulator images."""
    monkeypatch.setattr(SG, "CONV_FWD_V8", v8)
    torch.manual_seed(cin + cout + hw)
    cl = torch.channels_last
    ho = (hw - 1) // 2 + 1
    dy = torch.randn(n, cout, ho, ho, device=DEV).contiguous(memory_format=cl)
    w = (torch.randn(cout, cin, 3, 3, device=DEV) / (3 * cout ** 0.5)).contiguous(memory_format=cl)
    shape = (n, cin, hw, hw)
    assert SG.conv_dgrad_s2_ok(dy, w, shape)
    dx = SG.conv_dgrad_s2(dy, w, shape)
    ref = torch.nn.grad.conv2d_input(shape, w.double(), dy.double(), stride=2, padding=1)
    bound = torch.nn.grad.conv2d_input(shape, w.double().abs(), dy.double().abs(), stride=2, padding=1)
    assert dx.is_contiguous(memory_format=cl)
    err = ((dx.double() - ref).abs() / (bound + 1e-30)).max().item()
    assert err < (4e-7 if v8 else 2e-7), err


@pytest.mark.parametrize("M,K,N,splits,tile,variant", [(768, 8192, 768, 12, 0, 0), (2304, 8192, 768, 7, 0, 0),
                                                       (260, 1024, 196, 1, 0, 0), (256, 4096, 192, 3, 7, 0),
                                                       (128, 64, 128, 1, 0, 0), (2304, 8192, 768, 7, 0, 8),
                                                       (260, 1024, 196, 1, 0, 8), (768, 4096, 260, 12, 0, 8),
                                                       (256, 4096, 192, 3, 7, 8)])
def test_fused_row_sums(M, K, N, splits, tile, variant):
    """row_sums += a.sum(1) from the A staging of a weight-gradient GEMM (K-major a = dY^T), with
    and without split-K, ragged M, next to the accumulated product."""
    torch.manual_seed(M + K)
    dy = torch.randn(K, M, device=DEV)
    x = torch.randn(K, N, device=DEV)
    a = dy.t()
    c0 = torch.randn(M, N, device=DEV)
    c = c0.clone()
    rs0 = torch.randn(M, device=DEV)
    rs = rs0.clone()
    assert SG.row_sums_ok(a, rs, tile, variant)
    SG.matmul(a, x, out=c, accumulate=True, tile=tile, splits=splits, variant=variant, row_sums=rs)
    ref = a.double() @ x.double() + c0.double()
    assert ((c.double() - ref).abs() / (_bound(a, x) + 1)).max().item() < (4e-7 if variant == 8 else 2e-7)
    rref = dy.double().sum(0) + rs0.double()
    rbound = dy.double().abs().sum(0) + 1
    assert ((rs.double() - rref).abs() / rbound).max().item() < 1e-6
