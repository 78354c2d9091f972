"""1x1 convolutions as GEMMs (ops/conv1x1.py) against F.conv2d: forward, input gradient and
the weight gradient accumulated into the flat bf16 buffer by the split-K MFMA kernel."""
import pytest
import torch
import torch.nn.functional as F

from vodascheduler_amd.ops.conv1x1 import Conv1x1


def test_conv1x1_cpu_falls_back_to_conv2d():
    m = Conv1x1(16, 32, stride=2)
    x = torch.randn(2, 16, 8, 8)
    torch.testing.assert_close(m(x), F.conv2d(x, m.weight, stride=2))
    assert isinstance(m, torch.nn.Conv2d) and m.bias is None
    assert set(m.state_dict()) == {"weight"}


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / b.norm())


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,stride,hw", [(256, 64, 1, 14), (128, 512, 1, 7), (512, 1024, 2, 14),
                                               (1024, 256, 1, 7)])
def test_conv1x1_gemm_matches_conv2d(cin, cout, stride, hw):
    from vodascheduler_amd.ops.optim import make_optimizer

    torch.manual_seed(0)
    m = Conv1x1(cin, cout, stride=stride).cuda().to(memory_format=torch.channels_last).bfloat16()
    ref_w = m.weight.detach().float().clone().requires_grad_(True)
    opt = make_optimizer("sgd", m.parameters(), lr=0.0)  # flat grads: direct accumulation path
    x = torch.randn(4, cin, hw, hw, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    xr = x.float().detach().requires_grad_(True)
    xg = x.detach().requires_grad_(True)
    assert m._gemm_ok(xg)
    opt.zero_grad()
    y = m(xg)
    assert y.is_contiguous(memory_format=torch.channels_last)
    y_ref = F.conv2d(xr, ref_w, stride=stride)
    assert _rel(y, y_ref) < 1e-2
    g = torch.randn_like(y_ref)
    y.backward(g.bfloat16().to(memory_format=torch.channels_last))
    y_ref.backward(g)
    assert _rel(xg.grad, xr.grad) < 1e-2
    assert _rel(m.weight.grad, ref_w.grad) < 1e-2
    # a second backward accumulates (beta = 1), as autograd does
    m(xg).backward(g.bfloat16().to(memory_format=torch.channels_last))
    assert _rel(m.weight.grad, 2 * ref_w.grad) < 1e-2


@pytest.mark.gpu
def test_resnet50_uses_gemm_path_and_trains():
    from vodascheduler_amd.models import get_workload, prepare_model
    from vodascheduler_amd.ops.optim import make_optimizer

    w = get_workload("resnet50")
    torch.manual_seed(0)
    m = prepare_model(w, torch.device("cuda", 0))
    opt = make_optimizer(w.optimizer, m.parameters(), **w.opt_kwargs)
    x, y = w.make_batch(8, torch.device("cuda", 0), None)
    x = x.to(memory_format=torch.channels_last)
    n_gemm = sum(1 for mod in m.modules() if isinstance(mod, Conv1x1) and mod.in_channels >= 128)
    assert n_gemm >= 20
    losses = []
    for _ in range(4):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = w.loss(m, (x, y))
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert all(torch.isfinite(torch.tensor(losses))) and losses[-1] < losses[0], losses
