"""Fused cross-entropy (ops/xent.py) and flat-gradient embedding (ops/embedding.py) on CPU:
the PyTorch paths they fall back to here must equal the stock ops (the HIP kernels are
checked against the same references in tests/test_xent_gpu.py)."""
import torch
import torch.nn.functional as F

from vodascheduler_amd.ops.embedding import FusedEmbedding
from vodascheduler_amd.ops.optim import FusedAdamW
from vodascheduler_amd.ops.xent import softmax_cross_entropy
from vodascheduler_amd.utils.flat import grad_of


def test_xent_reference_matches_cross_entropy_with_padding_and_ignore():
    torch.manual_seed(0)
    x = torch.randn(37, 72, requires_grad=True)
    y = torch.randint(0, 70, (37,))
    y[::5] = 0
    loss, correct, n = softmax_cross_entropy(x, y, num_classes=70, ignore_index=0)
    ref = F.cross_entropy(x[:, :70], y, ignore_index=0)
    torch.testing.assert_close(loss, ref)
    valid = y != 0
    assert int(n) == int(valid.sum())
    assert int(correct) == int(((x[:, :70].argmax(1) == y) & valid).sum())
    loss.backward()
    g = x.grad.clone()
    x.grad = None
    ref.backward()
    torch.testing.assert_close(g, x.grad)
    assert float(g[:, 70:].abs().max()) == 0.0  # padding columns get no gradient


def test_fused_embedding_matches_nn_embedding():
    torch.manual_seed(0)
    ref = torch.nn.Embedding(50, 16)
    m = FusedEmbedding(50, 16)
    m.load_state_dict(ref.state_dict())
    ids = torch.randint(0, 50, (4, 9))
    ids[0, :3] = 7  # repeated tokens accumulate
    dy = torch.randn(4, 9, 16)
    (m(ids) * dy).sum().backward()
    (ref(ids) * dy).sum().backward()
    torch.testing.assert_close(m.weight.grad, ref.weight.grad)


def test_fused_embedding_scatters_into_flat_gradient():
    torch.manual_seed(0)
    m = FusedEmbedding(50, 16)
    ref = torch.nn.Embedding(50, 16)
    ref.load_state_dict(m.state_dict())
    opt = FusedAdamW(m.parameters(), lr=1e-3)
    opt.zero_grad()
    ids = torch.randint(0, 50, (3, 5))
    dy = torch.randn(3, 5, 16)
    (m(ids) * dy).sum().backward()
    (ref(ids) * dy).sum().backward()
    torch.testing.assert_close(grad_of(m.weight), ref.weight.grad)


def test_add_rows_gradients_match_broadcast_add():
    from vodascheduler_amd.ops.embedding import add_rows

    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.randn(2, 16))
    wr = torch.nn.Parameter(w.detach().clone())
    x = torch.randn(3, 5, 16, requires_grad=True)
    xr = x.detach().clone().requires_grad_(True)
    dy = torch.randn(3, 5, 16)
    (add_rows(x, w, 0) * dy).sum().backward()
    ((xr + wr[0]) * dy).sum().backward()
    torch.testing.assert_close(w.grad, wr.grad)
    torch.testing.assert_close(x.grad, xr.grad)
    # flat fp32 gradient path (the trainer's): accumulated into the row's slot
    opt = FusedAdamW([w], lr=1e-3)
    opt.zero_grad()
    (add_rows(x, w, 1) * dy).sum().backward()
    ref = torch.zeros(2, 16)
    ref[1] = dy.reshape(-1, 16).sum(0)
    torch.testing.assert_close(grad_of(w), ref)


def test_add_rows_position_block():
    from vodascheduler_amd.ops.embedding import add_rows

    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.randn(8, 16))
    wr = torch.nn.Parameter(w.detach().clone())
    x = torch.randn(3, 5, 16)
    dy = torch.randn(3, 5, 16)
    (add_rows(x, w, 0, 5) * dy).sum().backward()
    ((x + wr[:5][None]) * dy).sum().backward()
    torch.testing.assert_close(w.grad, wr.grad)
    opt = FusedAdamW([w], lr=1e-3)
    opt.zero_grad()
    (add_rows(x, w, 0, 5) * dy).sum().backward()
    torch.testing.assert_close(grad_of(w), wr.grad)
