"""fp32 GEMM at fp32 accuracy on the bf16 matrix cores (csrc/hip/splitgemm.hip).

gfx950 has no xf32 MFMA; its f32-input MFMA runs at the fp32 vector rate (157 TF), which is
where hipBLASLt's fp32 GEMMs (and the round-5 own f32-MFMA kernels) stop.  The kernel here
splits every fp32 operand exactly into three bf16 planes while staging it
(``x == hi + mid + lo``), multiplies the six significant cross products on
``v_mfma_f32_32x32x16_bf16`` and accumulates in fp32: fp32 accuracy at up to 16/6 of the fp32
MFMA rate.  ``split3`` / ``emulate`` below are the bit-exact host model of that arithmetic
(products of bf16 values are exact, so fp64 accumulation of the kept products reproduces the
kernel up to fp32 accumulation order), used by the CPU numerics tests.

    matmul(a, b)         a [M, K], b [K, N] fp32 (either may be a transposed view)
    linear(x, w, bias)   x [..., K] . w[N, K]^T + bias      (F.linear)

Reference: the fp32 Dense / EinsumDense projections of
examples/py/tensorflow2/neural_machine_translation_with_transformer.py:191-315 and the
fp32 Conv2D of tensorflow2_keras_cifar_elastic.py:148-158 (no mixed-precision policy).
"""
from __future__ import annotations

import os

import torch

from . import _native as N

EPI_NONE, EPI_GELU, EPI_DGELU = 0, 1, 2
TILES = {0: (128, 128), 1: (256, 128), 2: (128, 256), 5: (64, 256), 6: (256, 64), 7: (128, 96), 8: (64, 192)}


def thin_tile(M: int, Nn: int) -> int:
    """The tile for an M x N output with one 64-wide dimension (ResNet-50 stage-1 1x1 weight
    gradients: [64][256] / [256][64]), so that no 128-wide tile runs half empty; else tile 0."""
    if M == 64 and Nn % 256 == 0:
        return 5
    if Nn == 64 and M % 256 == 0:
        return 6
    return 0
# 0 = 6 products with the hi.hi products in their own accumulator (shipped); 1 = 6 products, one
# accumulator, software-pipelined split; 2 = 9 products; 3 = 3 products (~16-bit: error study
# only); 4 = 0 software-pipelined at one wave per SIMD (A/B)
VARIANT_NAMES = {0: "bf16x3-6p-dual", 1: "bf16x3-6p-single-pipe", 2: "bf16x3-9p-dual", 3: "bf16x2-3p-dual",
                 4: "bf16x3-6p-dual-pipe-1wave", 5: "bf16x3-6p-dual-product-outer",
                 6: "bf16x3-6p-dual-wavespec", 7: "bf16x3-6p-single-wavespec-lead2", 8: "bf16x3-6p-single-3wg"}
GEMM_MATH = VARIANT_NAMES[0]

# VODA_SPLIT_GEMM=0 routes the fp32 projections back to hipBLASLt (A/B switch)
ENABLED = os.environ.get("VODA_SPLIT_GEMM", "1") != "0"
# math / kernel variant of the Linear GEMMs (VARIANT_NAMES) and of the convolution weight
# gradient (0 one-role kernel, 1 / 2 wave-specialised, staging one / two stages ahead)
DEFAULT_VARIANT = 0
CONV_WGRAD_WS = 0
# 3x3 convolution weight gradients on the 128 x 128 tile with one accumulator at three workgroups
# per CU (the conv-gather image of variant 8; A/B switch)
CONV_WGRAD_V8 = True
# ... split-K towards two rounds of its 768 resident workgroups (1536) instead of 1024: C = 128 /
# 256 / 512 layers 388 -> 374, 379 -> 372, 395 -> 393 us (profiles/r6/resnet50_wgrad_splits_v8_probe.jsonl)
CONV_WGRAD_V8_ROUNDS = True
# the implicit-GEMM convolution forward (ResNet's stride-2 3x3 layers) and the polyphase input
# gradient's class GEMMs in the same form (A/B switch)
CONV_FWD_V8 = True
USE_T7 = True  # the 128 x 96 tile in ``choose`` (A/B switch)
# GEMMs whose B operand is K-major (input and weight gradients) on variant 8: one accumulator at
# three workgroups per CU (K-major B images leave room for three in LDS); qkv / fc1 / fc2 input
# gradients 184 -> 177, 239 -> 227, 246 -> 230 us, qkv weight gradient 183 -> 176 us
# (profiles/r6/splitgemm_v8_3wg_probe.jsonl); error still below hipBLASLt fp32's (A/B switch)
USE_V8_KMAJOR_B = True
# ... and the forwards (K-contiguous B) once the 96-B K-contiguous images fit three workgroups:
# qkv / fc1 / fc2 forwards 199 -> 192, 266 -> 250, 241 -> 235 us (profiles/r6/fwd_probe_kc96.jsonl)
USE_V8_FWD = True
# ... with 128 x 96 tiles where those fill whole rounds of 768 and 128 x 128 ones do not: the
# qkv forward ran 189.7 vs 188.9 us and the step tied (32.11 / 32.11 ms, profiles/r6/
# ab_t7_v8_bert_fp32.jsonl), so off; the tile-7 variant-8 image stays tested (A/B switch)
USE_T7_V8 = False
# a Linear's bias gradient summed in the weight-gradient GEMM's A staging (matmul(row_sums=...))
# instead of a separate column-sum pass over dY (A/B switch)
USE_FUSED_ROW_SUMS = True
# split-K reduce: slab groups per float4 column (-1 automatic: ~4096 blocks-worth of groups, >= 16
# slabs per group; 1 = one thread per column, the round-5 form)
REDUCE_GROUPS = -1
REDUCE_GROUPS_AUTO = True  # False: one group (A/B switch)
# K-contiguous operands staged with a row map whose 8-byte LDS writes hit 32 distinct banks per
# 16-lane group (csrc/hip/splitgemm.hip sx_kc_unit; False: consecutive rows, 2-way conflicts).
# Applies to the padded 112-B layout only (-DSX_KC_PITCH=112); the shipped 96-B layout's
# consecutive-row staging is the conflict-free one, and the kernel ignores this switch there.
WRITE_MAP = True
_applied = {"reduce_groups": None, "write_map": None}


def _sync_knobs(h) -> None:
    g = REDUCE_GROUPS if REDUCE_GROUPS_AUTO else 1
    if _applied["reduce_groups"] != g:
        h.sgemm_set_reduce_groups(int(g))
        _applied["reduce_groups"] = g
    if _applied["write_map"] != WRITE_MAP:
        h.sgemm_set_write_map(int(bool(WRITE_MAP)))
        _applied["write_map"] = WRITE_MAP

_WS: dict[torch.device, torch.Tensor] = {}


def split3(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Exact 3-way bf16 split of an fp32 tensor (round-to-nearest each step), as fp32 tensors:
    hi + mid + lo == x for every finite x whose residuals stay normal."""
    x = x.float()
    hi = x.to(torch.bfloat16).float()
    r = x - hi
    mid = r.to(torch.bfloat16).float()
    lo = (r - mid).to(torch.bfloat16).float()
    return hi, mid, lo


_PRODUCTS = {6: ((0, 0), (0, 1), (1, 0), (0, 2), (2, 0), (1, 1)),
             9: ((0, 0), (0, 1), (1, 0), (0, 2), (2, 0), (1, 1), (1, 2), (2, 1), (2, 2)),
             3: ((0, 0), (0, 1), (1, 0))}


def emulate(a: torch.Tensor, b: torch.Tensor, nprod: int = 6) -> torch.Tensor:
    """Host model of the kernel's arithmetic: sum of the kept bf16 cross products of ``a @ b``,
    accumulated in fp64 (each product is exact; only the accumulation order differs from the
    GPU), returned in fp64."""
    pa, pb = split3(a), split3(b)
    out = None
    for i, j in _PRODUCTS[nprod]:
        t = pa[i].double() @ pb[j].double()
        out = t if out is None else out + t
    return out


def _layout(t: torch.Tensor, rows_dim_first: bool) -> tuple[bool, int] | None:
    """(kmajor, ld) of a 2-D operand, or None if neither orientation is dense in one dim.

    For ``a`` [M, K]: K-contiguous when stride(1) == 1, K-major when stride(0) == 1.
    For ``b`` [K, N]: K-contiguous (b = W^T of a [N, K] W) when stride(0) == 1, K-major when
    stride(1) == 1."""
    s0, s1 = t.stride()
    if rows_dim_first:  # a [M, K]
        if s1 == 1 and (t.shape[0] == 1 or s0 >= t.shape[1]):
            return False, s0
        if s0 == 1 and s1 >= t.shape[0]:
            return True, s1
    else:               # b [K, N]
        if s0 == 1 and s1 >= t.shape[0]:
            return False, s1
        if s1 == 1 and s0 >= t.shape[1]:
            return True, s0
    return None


def _aligned(t: torch.Tensor, ld: int) -> bool:
    return t.data_ptr() % 16 == 0 and ld % 4 == 0


def supported(a: torch.Tensor, b: torch.Tensor) -> bool:
    """True when ``a @ b`` can run on the split kernel (fp32 CUDA operands, K % 16 == 0,
    M, N % 4 == 0, one dense dimension with 16-byte rows per operand)."""
    if not (ENABLED and a.is_cuda and b.is_cuda and a.dtype == torch.float32 and b.dtype == torch.float32):
        return False
    if a.dim() != 2 or b.dim() != 2 or a.shape[1] != b.shape[0]:
        return False
    M, K = a.shape
    Nn = b.shape[1]
    if M == 0 or Nn == 0 or K == 0 or K % 16 or M % 4 or Nn % 4:
        return False
    la, lb = _layout(a, True), _layout(b, False)
    return la is not None and lb is not None and _aligned(a, la[1]) and _aligned(b, lb[1])


def choose(M: int, Nn: int, K: int, variant: int = 0) -> tuple[int, int]:
    """(tile, splits) for an M x N x K GEMM on the 128 x 128 tile (two workgroups per CU, 512
    resident).  From the MI355X sweep over the BERT-base shapes (profiles/r6/splitgemm_probe.md):
    >= 1024 output tiles run whole; 384-1023 tiles split K in two when K >= 2048 (the single
    384-workgroup round leaves CUs with one workgroup idle half the time); small outputs (weight
    gradients: 36-144 tiles) split K towards ~1152 workgroups with >= 256 k per split.  The same
    shapes serve every math variant (``variant`` is accepted for call-site symmetry)."""
    tiles = -(-M // 128) * -(-Nn // 128)
    if variant == 8:  # three workgroups per CU: 128 x 128 tiles, splits as below
        if USE_T7_V8 and Nn % 96 == 0 and K <= 2304 and M >= 4096 and tiles >= 1024:
            # 128 x 96 where it fills whole rounds of the 768 resident workgroups and 128 x 128
            # does not (BERT-base qkv forward: 1536 vs 1152 tiles)
            t7 = -(-M // 128) * (Nn // 96)

            def fill3(t: int) -> float:
                return t / (-(-t // 768) * 768)

            if fill3(t7) > 1.05 * fill3(tiles):
                return 7, 1
        if tiles >= 1024:
            return 0, 1
        if tiles >= 384:
            return 0, 2 if K >= 2048 else 1
        if 96 <= tiles <= 160 and K >= 7 * 512:
            return 0, 7
        if 24 <= tiles <= 48 and K >= 12 * 512:
            return 0, 12
        return 0, max(1, min(16 if tiles >= 16 else 1024, 1152 // tiles, K // 256))
    # 128 x 96 tiles where they fill whole rounds of the 512 resident workgroups and 128 x 128
    # tiles do not (BERT-base: 8192 x 2304 as 1536 tiles, 8192 x 768 as 512): qkv forward 200 ->
    # 192 us, o forward 76 -> 71, o input gradient 78 -> 71 (profiles/r6/splitgemm_t7_sweep.jsonl);
    # not for K > 2304, where 128 x 128 with split-K 2 stays ahead (fc1 / fc2 input gradient / fc2)
    if USE_T7 and Nn % 96 == 0 and K <= 2304 and M >= 4096:
        t7 = -(-M // 128) * (Nn // 96)

        def fill(t: int) -> float:
            return t / (-(-t // 512) * 512)

        if t7 >= 384 and fill(t7) > 1.05 * fill(tiles):
            return 7, 1
    if tiles >= 1024:
        return 0, 1
    if tiles >= 384:
        return 0, 2 if K >= 2048 else 1
    # small outputs with long reductions (weight gradients over the tokens): the split-K sweep of
    # the BERT-base shapes (profiles/r6/splitgemm_wgrad_splits.jsonl) put the optimum at 7 splits
    # for 108-144 output tiles (qkv 210 -> 183 us, fc1 / fc2 254 -> 237 us vs the ~1152-workgroup
    # rule below) and 12 for 36 tiles (o: 89 -> 74 us)
    if 96 <= tiles <= 160 and K >= 7 * 512:
        return 0, 7
    if 24 <= tiles <= 48 and K >= 12 * 512:
        return 0, 12
    # tiny outputs with huge reductions (ResNet 1x1 weight gradients: 64 x 256 over 800k pixels)
    # split further: the slabs stay small
    s = max(1, min(16 if tiles >= 16 else 1024, 1152 // tiles, K // 256))
    return 0, s


def _workspace(device: torch.device, floats: int) -> torch.Tensor:
    w = _WS.get(device)
    if w is None or w.numel() < floats:
        w = _WS[device] = torch.empty(max(floats, 1 << 20), dtype=torch.float32, device=device)
    return w


def matmul(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False,
           bias: torch.Tensor | None = None, epi: int = EPI_NONE, aux: torch.Tensor | None = None,
           tile: int | None = None, splits: int | None = None, variant: int | None = None,
           row_sums: torch.Tensor | None = None) -> torch.Tensor:
    """``out (+)= a @ b (+ bias)`` on the split kernel; epi GELU writes the pre-activation
    into ``aux`` and gelu of it into ``out``, epi DGELU multiplies by gelu'(aux).  ``row_sums``
    (fp32 [M], 16-B aligned; K-major ``a`` only, see ``row_sums_ok``): ``row_sums += a.sum(1)``
    from the A staging of the same launch (a Linear's bias gradient next to its weight gradient
    dW = dY^T X).  Callers check ``supported`` (CPU tensors get the PyTorch reference)."""
    M, K = a.shape
    Nn = b.shape[1]
    if not a.is_cuda:
        if row_sums is not None:
            row_sums.add_(a.float().sum(1))
        y = a.float() @ b.float()
        if accumulate and out is not None:
            y = y + out
        if bias is not None:
            y = y + bias.float()
        if epi == EPI_GELU:
            aux.copy_(y)
            y = torch.nn.functional.gelu(y, approximate="tanh")
        elif epi == EPI_DGELU:
            from .ffn import gelu_tanh_grad_ref

            y = y * gelu_tanh_grad_ref(aux)
        if out is None:
            return y
        out.copy_(y)
        return out
    la, lb = _layout(a, True), _layout(b, False)
    if la is None or lb is None:
        raise ValueError("splitgemm.matmul: operands need one dense dimension")
    if out is None:
        if accumulate:
            raise ValueError("splitgemm.matmul: accumulate needs out")
        out = torch.empty(M, Nn, dtype=torch.float32, device=a.device)
    if out.stride(1) != 1 or out.shape != (M, Nn):
        raise ValueError("splitgemm.matmul: out must be [M, N] with unit column stride")
    if variant is None:
        variant = plan_variant(lb[0], tile, M, Nn, K)
    t0, s0 = choose(M, Nn, K, variant)
    tile = t0 if tile is None else tile
    splits = s0 if splits is None else splits
    if variant == 8 and tile not in (0, 7):  # variant 8 exists on the 128 x 128 / 128 x 96 tiles
        variant = DEFAULT_VARIANT
    if row_sums is not None and not row_sums_ok(a, row_sums, tile, variant):
        raise ValueError("splitgemm.matmul: row_sums need a K-major a, tile 0 / 7, variant 0 / 8 and an aligned fp32 [M]")
    h = N.hip()
    _sync_knobs(h)
    ws_floats = h.sgemm_f32_workspace_floats(M, Nn, splits)
    ws = _workspace(a.device, ws_floats) if ws_floats else None
    if bias is not None:
        bias = bias.float().contiguous()
    ld_aux = 0
    if aux is not None:
        if aux.dtype != torch.float32 or aux.stride(1) != 1 or aux.shape != (M, Nn):
            raise ValueError("splitgemm.matmul: aux must be fp32 [M, N] with unit column stride")
        ld_aux = aux.stride(0)
    h.sgemm_f32(a.data_ptr(), la[1], la[0], b.data_ptr(), lb[1], lb[0], out.data_ptr(), out.stride(0), M, Nn, K,
                bool(accumulate), bias.data_ptr() if bias is not None else 0, int(epi),
                aux.data_ptr() if aux is not None else 0, ld_aux, int(tile), int(splits), int(variant),
                ws.data_ptr() if ws is not None else 0, ws.numel() if ws is not None else 0, N.stream_of(a),
                row_sums.data_ptr() if row_sums is not None else 0)
    return out


def plan_variant(b_kmajor: bool, tile: int | None = None, M: int = 0, Nn: int = 0, K: int = 0) -> int:
    """The math / kernel variant ``matmul`` runs when the caller does not pin one: variant 8 (one
    accumulator, three workgroups per CU) for K-major B operands (``USE_V8_KMAJOR_B``) and, since
    the 96-B K-contiguous LDS layout lets three workgroups fit, for K-contiguous ones too
    (``USE_V8_FWD``); else ``DEFAULT_VARIANT``.  Shapes whose variant-0 plan is a whole round of
    128 x 96 tiles stay there when variant 8 would leave its 768-workgroup round half empty
    (BERT-base o forward / input gradient: 73 vs 78-81 us, profiles/r6/splitgemm_v8_3wg_probe.jsonl)."""
    if tile is not None or DEFAULT_VARIANT != 0 or not (USE_V8_KMAJOR_B if b_kmajor else USE_V8_FWD):
        return DEFAULT_VARIANT
    if M and choose(M, Nn, K, 0)[0] == 7:
        t, sp = choose(M, Nn, K, 8)
        if -(-M // 128) * -(-Nn // 128) * sp < 768:
            return DEFAULT_VARIANT
    return 8


def plan(a: torch.Tensor, b: torch.Tensor) -> tuple[int, int, int]:
    """(tile, splits, variant) ``matmul(a, b)`` picks for these operands."""
    lb = _layout(b, False)
    M, K, Nn = a.shape[0], a.shape[1], b.shape[1]
    v = plan_variant(bool(lb and lb[0]), None, M, Nn, K)
    t, sp = choose(M, Nn, K, v)
    return t, sp, v


def row_sums_ok(a: torch.Tensor, row_sums: torch.Tensor, tile: int, variant: int) -> bool:
    """Can ``matmul`` fuse ``row_sums += a.sum(1)`` on this launch shape?  K-major a (a weight
    gradient's dY^T), tile 0 or 7, math variant 0 or 8, a contiguous
    16-byte-aligned fp32 [M] target."""
    if not USE_FUSED_ROW_SUMS or not a.is_cuda:
        return False
    la = _layout(a, True)
    M = a.shape[0]
    shape_ok = tile in (0, 7) and variant in (0, 8)
    return (la is not None and la[0] and shape_ok and row_sums.dtype == torch.float32
            and row_sums.is_cuda and row_sums.dim() == 1 and row_sums.numel() == M and row_sums.is_contiguous()
            and row_sums.data_ptr() % 16 == 0)


def linear(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """``F.linear(x, w, bias)`` in fp32 on the split kernel (x [..., K], w [N, K])."""
    x2 = x.reshape(-1, x.shape[-1])
    y = matmul(x2, w.t(), bias=bias)
    return y.view(*x.shape[:-1], w.shape[0])


def conv_wgrad_ok(dy: torch.Tensor, x: torch.Tensor, gw: torch.Tensor) -> bool:
    """Does the implicit-GEMM convolution weight gradient take these fp32 operands?  dy
    [N, Cout, Ho, Wo] and x [N, Cin, H, W] channels_last, gw the channels_last filter gradient
    [Cout, Cin, KH, KW] (memory [Cout][KH][KW][Cin])."""
    cl = torch.channels_last
    if not (ENABLED and dy.is_cuda and x.is_cuda and gw.is_cuda):
        return False
    if not (dy.dtype == x.dtype == gw.dtype == torch.float32 and dy.dim() == x.dim() == gw.dim() == 4):
        return False
    if not (dy.is_contiguous(memory_format=cl) and x.is_contiguous(memory_format=cl)
            and gw.is_contiguous(memory_format=cl)):
        return False
    n, cin = x.shape[:2]
    cout = gw.shape[0]
    if gw.shape[1] != cin or dy.shape[0] != n or dy.shape[1] != cout or cin % 4 or cout % 4:
        return False
    if (n * dy.shape[2] * dy.shape[3]) % 16:
        return False
    return dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0 and gw.data_ptr() % 16 == 0


def conv_wgrad_splits(cout: int, n_cols: int, pixels: int, tile: int = 0, target: int = 1024) -> int:
    """Split-K count of a convolution weight gradient: ~``target`` workgroups, >= 256 pixels per
    split.  1024 (two rounds of the 512 resident 128 x 128 workgroups) for the 3x3 implicit GEMMs;
    the 1x1 weight gradients pass 512: one round ran all nine ResNet-50 1x1 shapes 5-11 % faster
    than two (profiles/r6/resnet50_wgrad_splits_probe_b.jsonl)."""
    bm, bn = TILES[tile]
    tiles = -(-cout // bm) * -(-n_cols // bn)
    return max(1, min(max(1, target // tiles), pixels // 256))


def conv_wgrad_tile(cout: int, n_cols: int) -> int:
    """Tile of a convolution weight gradient [Cout][KH*KW*Cin]: 64 x 192 for the 64-channel 3x3
    layers (576 columns = 3 tiles exactly), 128 x 128 otherwise."""
    return 8 if cout == 64 and n_cols % 192 == 0 else 0


def conv_wgrad_(dy: torch.Tensor, x: torch.Tensor, gw: torch.Tensor, stride: int, padding: int,
                accumulate: bool = True, splits: int | None = None, tile: int | None = None) -> None:
    """``gw (+)= dW`` of a convolution on the split-bf16 MFMA kernel (callers check
    ``conv_wgrad_ok``); CPU tensors get the fp32 reference."""
    if not dy.is_cuda:
        w = torch.nn.grad.conv2d_weight(x.float(), gw.shape, dy.float(), stride=stride, padding=padding)
        gw.copy_(w + gw if accumulate else w)
        return
    n, cin, H, W = x.shape
    cout, _, kh, kw = gw.shape
    ho, wo = dy.shape[2], dy.shape[3]
    tile = conv_wgrad_tile(cout, kh * kw * cin) if tile is None else tile
    v8 = CONV_WGRAD_V8 and CONV_WGRAD_WS == 0 and tile == 0
    target = 1536 if v8 and CONV_WGRAD_V8_ROUNDS else 1024
    s = conv_wgrad_splits(cout, kh * kw * cin, n * ho * wo, tile, target) if splits is None else splits
    h = N.hip()
    _sync_knobs(h)
    h.sgemm_conv_wgrad_set_ws(3 if v8 else CONV_WGRAD_WS)
    ws_floats = h.sgemm_f32_workspace_floats(cout, kh * kw * cin, s)
    ws = _workspace(dy.device, ws_floats) if ws_floats else None
    h.sgemm_conv_wgrad_f32(dy.data_ptr(), x.data_ptr(), gw.data_ptr(), n, H, W, cin, ho, wo, cout, kh, kw,
                           int(stride), int(padding), s, bool(accumulate), ws.data_ptr() if ws is not None else 0,
                           ws.numel() if ws is not None else 0, N.stream_of(dy), int(tile))


def conv_fwd_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Does the implicit-GEMM convolution forward take these fp32 operands?  x [N, Cin, H, W] and
    w [Cout, Cin, KH, KW], both channels_last, Cin % 16 == 0, Cout % 4 == 0."""
    cl = torch.channels_last
    if not (ENABLED and x.is_cuda and w.is_cuda and x.dtype == w.dtype == torch.float32):
        return False
    if x.dim() != 4 or w.dim() != 4 or w.shape[1] != x.shape[1] or x.shape[1] % 16 or w.shape[0] % 4:
        return False
    if not (x.is_contiguous(memory_format=cl) and w.is_contiguous(memory_format=cl)):
        return False
    return x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0


def conv_fwd(x: torch.Tensor, w: torch.Tensor, stride: int, padding: int) -> torch.Tensor:
    """``F.conv2d(x, w, None, stride, padding)`` for fp32 channels_last operands (callers check
    ``conv_fwd_ok``) as one implicit GEMM on the split-bf16 MFMA kernel; channels_last output.
    CPU tensors get the PyTorch reference."""
    if not x.is_cuda:
        return torch.nn.functional.conv2d(x, w, None, stride, padding)
    n, cin, H, W = x.shape
    cout, _, kh, kw = w.shape
    ho = (H + 2 * padding - kh) // stride + 1
    wo = (W + 2 * padding - kw) // stride + 1
    y = torch.empty((n, cout, ho, wo), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
    _sync_knobs(N.hip())
    N.hip().sgemm_conv_fwd_set_v8(int(CONV_FWD_V8))
    N.hip().sgemm_conv_fwd_f32(x.data_ptr(), w.data_ptr(), y.data_ptr(), n, H, W, cin, ho, wo, cout, kh, kw,
                               int(stride), int(padding), N.stream_of(x))
    return y


_S2_TAPS = {0: (1,), 1: (2, 0)}  # kernel rows (cols) of the taps that reach even / odd input rows


def conv_dgrad_s2_ok(dy: torch.Tensor, w: torch.Tensor, in_shape) -> bool:
    """Input gradient of a stride-2, pad-1 3x3 fp32 convolution on the polyphase implicit GEMMs?"""
    cl = torch.channels_last
    if not (ENABLED and dy.is_cuda and w.is_cuda and dy.dtype == w.dtype == torch.float32):
        return False
    if dy.dim() != 4 or w.dim() != 4 or tuple(w.shape[2:]) != (3, 3) or len(in_shape) != 4:
        return False
    n, cin, H, W = in_shape
    cout = w.shape[0]
    if w.shape[1] != cin or dy.shape[1] != cout or dy.shape[0] != n or cout % 16 or cin % 4:
        return False
    if dy.shape[2] != (H - 1) // 2 + 1 or dy.shape[3] != (W - 1) // 2 + 1:
        return False
    return dy.is_contiguous(memory_format=cl) and dy.data_ptr() % 16 == 0


def conv_dgrad_s2(dy: torch.Tensor, w: torch.Tensor, in_shape) -> torch.Tensor:
    """dX of ``conv2d(x, w, stride=2, padding=1)`` (3x3, fp32, channels_last) as four polyphase
    implicit GEMMs on the split-bf16 MFMA kernel: the input pixels of one (row, column) parity
    class receive 1, 2, 2 or 4 of the nine taps, each a stride-1 gather of dY (no zero-inserted
    map, no wasted products).  CPU tensors get the PyTorch reference."""
    n, cin, H, W = in_shape
    if not dy.is_cuda:
        return torch.nn.grad.conv2d_input(tuple(in_shape), w, dy, stride=2, padding=1)
    cout = w.shape[0]
    ho, wo = dy.shape[2], dy.shape[3]
    dx = torch.empty((n, cin, H, W), dtype=torch.float32, device=dy.device, memory_format=torch.channels_last)
    wt = w.permute(2, 3, 0, 1)  # [kh][kw][co][ci] view
    h = N.hip()
    _sync_knobs(h)
    h.sgemm_conv_fwd_set_v8(int(CONV_FWD_V8))  # the class GEMMs take the forward's kernel form
    st = N.stream_of(dy)
    for ph in (0, 1):
        for pw in (0, 1):
            if (H - ph + 1) // 2 <= 0 or (W - pw + 1) // 2 <= 0:
                continue
            wc = torch.stack([wt[kh, kw] for kh in _S2_TAPS[ph] for kw in _S2_TAPS[pw]]).contiguous()
            h.sgemm_conv_dgrad_s2_class(dy.data_ptr(), wc.data_ptr(), dx.data_ptr(), n, ho, wo, cout, H, W, cin,
                                        ph, pw, st)
    return dx
