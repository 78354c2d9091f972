"""Pre-tuned fp32 library GEMMs (utils/tunable.py): the shipped TunableOp results load with
tuning off, a tuned shape computes the same product as fp64, and an untuned shape still runs
(the library default)."""
import os

import pytest
import torch

from vodascheduler_amd.utils import tunable

pytestmark = pytest.mark.gpu


@pytest.mark.skipif(not os.path.exists(tunable.results_path("fp32")), reason="no shipped fp32 results")
def test_shipped_fp32_results_load_and_compute_correctly():
    assert tunable.configure("fp32")
    st = tunable.status()
    assert st["enabled"] and not st["tuning"] and st["entries"] > 0
    torch.manual_seed(0)
    x = torch.randn(8192, 768, device="cuda")
    w = torch.randn(2304, 768, device="cuda") * 0.05   # BERT-base QKV projection, a tuned shape
    b = torch.randn(2304, device="cuda")
    y = torch.nn.functional.linear(x, w, b)
    ref = torch.nn.functional.linear(x.double(), w.double(), b.double())
    assert float((y.double() - ref).norm() / ref.norm()) < 1e-5
    z = torch.randn(333, 77, device="cuda") @ torch.randn(77, 129, device="cuda")  # not in the file
    assert z.shape == (333, 129) and torch.isfinite(z).all()
