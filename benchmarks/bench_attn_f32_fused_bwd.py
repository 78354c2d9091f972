"""fp32 attention forward + backward on BERT-base's shape (B 64, H 12, T 128, D 64): the
one-workgroup-per-head fused backward (mode 1, default) vs the dQ + dK/dV passes (mode 0),
interleaved, CUDA-event timed (per call, forward included).

python benchmarks/bench_attn_f32_fused_bwd.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import _native  # noqa: E402
from vodascheduler_amd.ops.attention import attention_qkvpacked  # noqa: E402

h = _native.hip()
B, H, T, D = 64, 12, 128, 64
qkv = torch.randn(B, T, 3, H, D, device="cuda", requires_grad=True)
do = torch.randn(B, T, H, D, device="cuda")


def run():
    o = attention_qkvpacked(qkv, None, False, D ** -0.5)
    o.backward(do)


res = {}
try:
    for rep in range(3):
        for mode in (0, 1):
            h.attn_f32_set_fused_bwd(mode)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                run()
            e.record()
            torch.cuda.synchronize()
            res.setdefault(str(mode), []).append(round(s.elapsed_time(e) / 20 * 1e3, 1))
finally:
    h.attn_f32_set_fused_bwd(1)
print(json.dumps({"shape": [B, H, T, D], "fwd_plus_bwd_us": res, "modes": {"0": "two-pass", "1": "fused"}}))
