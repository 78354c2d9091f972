"""Linear-layer weight gradient (+ fused bias gradient) on the split-K MFMA kernel of
csrc/hip/wgrad.hip, with the fp32 PyTorch reference of the same op.

    dW (+)= dY^T X        db (+)= dY.sum(0)        dY [M, N], X [M, K], dW [N, K], db [N]

These are the "reduction over tokens" GEMMs of every Linear backward (BERT-base: M = 8192
tokens); ``ops/dense.py`` routes them here when the layer accumulates straight into the
optimizer's flat gradient buffer -- fp32 by default (the kernel rounds its fp32 MFMA
accumulators once into the fp32 gradient), bf16 when low-precision gradients were chosen.
"""
from __future__ import annotations

import math
import os

import torch

from . import _native as N

TILE = 128
# 0: register-staged LDS double buffer; 1 / 2 / 3: LDS ring of 4 / 2 / 3 stages of 64 tokens
# filled by global_load_lds; 4 / 5: ring of 4 / 5 stages of 32 tokens; 6 / 7 / 8: 256 x 256
# tile, 8 waves, ring of 4 x 32 / 5 x 32 / 3 x 32 tokens; 9 / 10: 256 x 256 tile on two
# 64-token stages (128 KB) / three 48-token stages (144 KB); 11 / 12: fill-only probes of 9 / 10
# (no MFMA, dW undefined: benchmarks only).  Default 2 (64 KB ring, 2 workgroups per CU): fastest in the BERT-base step
# on MI355X (profiles/r1_wgrad_v3.md)
VARIANT = 2
# _VARIANT_FIXED = True: VARIANT for every shape (benchmarks); otherwise tall
# convolution-sized reductions use the deeper LDS rings at half the default split count
# (per-shape sweep on MI355X, fp32 output, profiles/raw/r2_wgrad_variant_split_sweep.jsonl:
# ResNet-50 stage 1 (M = 802816) 150-155 -> 131-137 us with variant 1, stage 2 (M = 200704)
# 95-96 -> 79 us with variant 3, and variant 1 once the block order became split-major;
# stages 3-4 and the BERT shapes gain nothing)
_VARIANT_FIXED = False
# _WIDE = False: keep every shape on the 128 x 128 tile
_WIDE = True


def choose(M: int, N_: int, K: int) -> tuple[int, int]:
    """(variant, splits) for a weight-gradient GEMM of M reduction rows."""
    if _VARIANT_FIXED:
        return VARIANT, default_splits(M, N_, K, variant=VARIANT)
    if M < 150_000:
        # >= 16 tiles of 256 x 256 and >= 4096 tokens: the wide two-stage kernel (variant 9)
        # at one round of <= 256 workgroups; per-shape sweep on MI355X (BERT-base, fp32 dW,
        # profiles/r3/wgrad_v9_sweep.jsonl): qkv 60.7 -> 55.2 us, fc1 67.8 -> 62.8, fc2
        # 68.1 -> 62.4; the 768 x 768 projection (9 wide tiles) stays on the 128 x 128 tile
        if _WIDE and M >= 4096 and math.ceil(N_ / WIDE_TILE) * math.ceil(K / WIDE_TILE) >= 16:
            return 9, default_splits(M, N_, K, variant=9)
        return VARIANT, default_splits(M, N_, K, variant=VARIANT)
    # split-major block order re-sweep (profiles/raw/r2_wgrad_sweep_split_major.jsonl): the
    # 4-stage ring at half the default split count is best for stage 2 too (75-76 -> 72 us)
    return 1, max(1, default_splits(M, N_, K, variant=1) // 2)
_ZERO: dict[torch.device, torch.Tensor] = {}


def _zero_rows(device: torch.device) -> torch.Tensor:
    """16-byte-aligned zeros the LDS-DMA variant reads for token rows past a split."""
    z = _ZERO.get(device)
    if z is None:
        z = _ZERO[device] = torch.zeros(64, dtype=torch.bfloat16, device=device)
    return z


WIDE_TILE = 256  # variants 6-9: 256 x 256 outputs per workgroup, one workgroup per CU


def default_splits(M: int, N_: int, K: int, target_blocks: int | None = None, variant: int | None = None) -> int:
    """Split the token dimension until the grid is ~1.7 waves of workgroups on the 256 CUs
    (two fit per CU), keeping >= 4 k-stages of 64 tokens per split.  Measured optimum on
    MI355X for the BERT-base shapes (benchmarks/bench_wgrad.py, profiles/): 12 splits for
    768x768 (36 tiles), 4 for 2304x768, 3 for 3072x768 / 768x3072.  Convolution-sized token
    counts (ResNet 1x1 convs: 800k rows, 2-32 tiles) go up to 256 splits.  The wide-tile
    variants (one 512-thread workgroup per CU) aim at one wave of 256 workgroups."""
    v = VARIANT if variant is None else int(variant)
    tile = WIDE_TILE if v >= 6 else TILE
    if target_blocks is None:
        target_blocks = 256 if v >= 6 else 432
    tiles = math.ceil(N_ / tile) * math.ceil(K / tile)
    # wide tiles: one workgroup per CU, so the grid must not spill into a second round
    s = target_blocks // tiles if v >= 6 else math.ceil(target_blocks / tiles)
    return max(1, min(s, 256, M // 256 if M >= 256 else 1))


def supported(dy2: torch.Tensor, x2: torch.Tensor, gw: torch.Tensor, gb: torch.Tensor | None = None) -> bool:
    """True when the HIP kernel can run these operands (bf16 inputs, bf16 or fp32 dW/db,
    16-byte aligned rows)."""
    if not (dy2.is_cuda and x2.is_cuda and gw.is_cuda):
        return False
    if dy2.dtype != torch.bfloat16 or x2.dtype != torch.bfloat16 or gw.dtype not in (torch.bfloat16, torch.float32):
        return False
    if dy2.dim() != 2 or x2.dim() != 2 or gw.dim() != 2:
        return False
    M, N_ = dy2.shape
    K = x2.shape[1]
    if x2.shape[0] != M or tuple(gw.shape) != (N_, K) or M == 0 or N_ % 8 or K % 8:
        return False
    if dy2.stride(1) != 1 or x2.stride(1) != 1 or gw.stride(1) != 1:
        return False
    if dy2.stride(0) % 8 or x2.stride(0) % 8 or gw.stride(0) % 8:
        return False
    if dy2.data_ptr() % 16 or x2.data_ptr() % 16 or gw.data_ptr() % 16:
        return False
    if gb is not None and (gb.dtype != gw.dtype or not gb.is_contiguous() or gb.numel() != N_):
        return False
    return True


def wgrad_ref(dy2: torch.Tensor, x2: torch.Tensor, gw: torch.Tensor, gb: torch.Tensor | None = None,
              accumulate: bool = True) -> tuple[torch.Tensor, torch.Tensor | None]:
    """fp32 reference: returns the new (dW, db) in fp32 without touching the inputs."""
    w = dy2.float().t() @ x2.float()
    b = dy2.float().sum(0) if gb is not None else None
    if accumulate:
        w = w + gw.float()
        if b is not None:
            b = b + gb.float()
    return w, b


def wgrad_accumulate_(dy2: torch.Tensor, x2: torch.Tensor, gw: torch.Tensor, gb: torch.Tensor | None = None,
                      accumulate: bool = True, splits: int | None = None, variant: int | None = None) -> None:
    """``gw (+)= dy2^T x2`` and ``gb (+)= dy2.sum(0)`` in place (fp32 accumulation, one rounding)."""
    if not dy2.is_cuda:
        w, b = wgrad_ref(dy2, x2, gw, gb, accumulate)
        gw.copy_(w.to(gw.dtype))
        if gb is not None:
            gb.copy_(b.to(gb.dtype))
        return
    if not supported(dy2, x2, gw, gb):
        raise ValueError(f"wgrad: unsupported operands dy {tuple(dy2.shape)} {dy2.dtype} stride {dy2.stride()}, "
                         f"x {tuple(x2.shape)} {x2.dtype} stride {x2.stride()}, dw {tuple(gw.shape)} {gw.dtype}")
    M, N_ = dy2.shape
    K = x2.shape[1]
    if variant is None and splits is None:
        v, s = choose(M, N_, K)
    else:
        v = VARIANT if variant is None else int(variant)
        s = splits if splits is not None else default_splits(M, N_, K, variant=v)
    h = N.hip()
    nws = h.wgrad_workspace_floats(M, N_, K, s)
    ws = torch.empty(nws, dtype=torch.float32, device=dy2.device) if nws else None
    h.wgrad_gemm(dy2.data_ptr(), dy2.stride(0), x2.data_ptr(), x2.stride(0), gw.data_ptr(), gw.stride(0),
                 N.ptr(gb), M, N_, K, s, N.ptr(ws), bool(accumulate), _zero_rows(dy2.device).data_ptr(), v,
                 N.dtype_code(gw.dtype), N.stream_of(dy2))
