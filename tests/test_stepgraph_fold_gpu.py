"""Whole-step hipGraph replay of parameters whose gradient comes from stock autograd (the
bf16-weight / fp32-flat-gradient fold hook, utils/flat.py ``_fold_lowp_grad``): every replay
must reproduce the eager gradient, not only the first (BERT-base check 28: ``type_emb.weight``
lost its gradient from the second replay on)."""
import pytest
import torch

from vodascheduler_amd.models import cast_compute_weights_
from vodascheduler_amd.ops.optim import make_optimizer
from vodascheduler_amd.runtime.stepgraph import StepGraph
from vodascheduler_amd.utils.flat import grad_of

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


class _Net(torch.nn.Module):
    def __init__(self, d=64):
        super().__init__()
        self.emb = torch.nn.Embedding(4, d)           # used as a broadcast row: weight[0]
        self.lin = torch.nn.Linear(d, 64)             # stock autograd weight gradient
        self.out = torch.nn.Linear(64, 8)

    def forward(self, x):
        h = x + self.emb.weight[0]
        return self.out(torch.relu(self.lin(h)))


@pytest.mark.parametrize("opt_name,shape,dt", [("sgd", (512, 64), torch.float32), ("adamw", (512, 64), torch.float32),
                                               ("adamw", (64, 128, 768), torch.float32),
                                               ("adamw", (64, 128, 768), torch.bfloat16)])  # BERT-base shapes
def test_fold_path_gradients_survive_every_replay(opt_name, shape, dt):
    torch.manual_seed(0)
    m = cast_compute_weights_(_Net(shape[-1]).to(DEV))
    opt = make_optimizer(opt_name, m.parameters(), lr=0.0)
    x = torch.randn(*shape, device=DEV).to(dt)
    y = torch.randint(0, 8, shape[:-1], device=DEV)

    def step(b):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            loss = torch.nn.functional.cross_entropy(m(b[0]).float().reshape(-1, 8), b[1].reshape(-1))
        loss.backward()
        opt.step()
        return loss

    side = torch.cuda.Stream()
    for _ in range(3):
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step((x, y))
        torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    step((x, y))
    torch.cuda.synchronize()
    ref = {n: grad_of(p).float().clone() for n, p in m.named_parameters()}
    g = StepGraph(step, (x, y), m, opt)
    for r in range(4):
        g.replay((x, y))
        torch.cuda.synchronize()
        junk = [torch.randn(1 << 20, device=DEV) for _ in range(8)]  # eager work between replays
        del junk
        for n, p in m.named_parameters():
            torch.testing.assert_close(grad_of(p).float(), ref[n], rtol=1e-3, atol=1e-6,
                                       msg=lambda s, n=n, r=r: f"replay {r} {n}: {s}")
