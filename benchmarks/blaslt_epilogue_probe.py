"""Which hipBLASLt epilogues have bf16 kernels on this GPU (BERT-base FFN shapes)?

python benchmarks/blaslt_epilogue_probe.py   -> one JSON line per (epilogue, op(A), shape)
"""
import json
import os
import sys

import torch  # noqa: F401  (HIP runtime first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import _native  # noqa: E402

EPI = {"DEFAULT": 1, "RELU": 2, "BIAS": 4, "RELU_BIAS": 6, "GELU": 32, "GELU_BIAS": 36, "GELU_AUX": 160,
       "GELU_AUX_BIAS": 164, "DGELU": 192, "DGELU_BGRAD": 208, "BGRADA": 256, "BGRADB": 512}
h = _native.hip()
for name, e in EPI.items():
    for ta in (True, False):
        for (m, n, k) in ((3072, 8192, 768), (768, 8192, 3072)):
            print(json.dumps({"epilogue": name, "trans_a": ta, "m": m, "n": n, "k": k,
                              "algos": h.gemm_epilogue_algos(e, ta, m, n, k)}), flush=True)
