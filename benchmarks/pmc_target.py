"""Small fixed workload for hardware-counter checks (tests/test_pmc_gpu.py): the fp32 1x1
GEMM with BN statistics (conv1x1_f32.hip), the bf16 statistics GEMM (gemm_bnstats.hip) and
the fp32 fused attention forward (attention_f32.hip), a few launches each."""
import torch

from vodascheduler_amd.ops import _native as N
from vodascheduler_amd.ops.attention import fused_attention


def main() -> None:
    h = N.hip()
    torch.manual_seed(0)
    M, Nc, K = 65536, 256, 256
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(Nc, K, device="cuda") * 0.05
    y = torch.empty(M, Nc, device="cuda")
    G = h.gemm_f32_stats_groups(M, Nc, K)
    part = torch.empty(2 * G * Nc, device="cuda")
    xb, wb = x.bfloat16(), w.bfloat16()
    yb = torch.empty(M, Nc, dtype=torch.bfloat16, device="cuda")
    Kb = 128
    Gb = h.gemm_bnstats_groups(M, Nc, Kb)
    partb = torch.empty(2 * Gb * Nc, device="cuda")
    xb2, wb2 = xb[:, :Kb].contiguous(), wb[:, :Kb].contiguous()
    q = torch.randn(8, 12, 128, 64, device="cuda")
    for _ in range(3):
        h.gemm_f32_stats(x.data_ptr(), w.data_ptr(), y.data_ptr(), part.data_ptr(), M, Nc, K, G, N.stream_of(x),
                         False, False)
        h.gemm_bnstats(xb2.data_ptr(), wb2.data_ptr(), yb.data_ptr(), partb.data_ptr(), M, Nc, Kb, Gb,
                       N.stream_of(x), False)
        fused_attention(q, q, q)
    torch.cuda.synchronize()
    print("pmc target done")


if __name__ == "__main__":
    main()
