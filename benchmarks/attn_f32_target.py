"""fp32 fused attention at the BERT-base shape (B 64, H 12, T 128, D 64), forward + backward,
a few iterations: the target of hardware-counter passes on the attention_f32.hip kernels."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops.attention import fused_attention  # noqa: E402


def main() -> None:
    torch.manual_seed(0)
    q, k, v = (torch.randn(64, 12, 128, 64, device="cuda", requires_grad=True) for _ in range(3))
    mask = torch.ones(64, 128, dtype=torch.bool, device="cuda")
    mask[:, 120:] = False
    for _ in range(5):
        o = fused_attention(q, k, v, mask)
        o.backward(torch.ones_like(o))
    torch.cuda.synchronize()
    print("attention target done")


if __name__ == "__main__":
    main()
