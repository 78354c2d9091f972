"""HIP fused cross-entropy (csrc/hip/xent.hip), the split-K input gradient of vocab-sized
heads (ops/dense.py ``_dgrad``) and the flat-gradient embedding on MI355X, against plain
PyTorch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

from vodascheduler_amd.ops import _native
from vodascheduler_amd.ops.xent import _XentFn, softmax_cross_entropy, xent_ref

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("rows,ld,V,dtype,ignore", [
    (1280, 30528, 30522, torch.bfloat16, -100),   # BERT-base MLM head (padded vocab)
    (2048, 15000, 15000, torch.bfloat16, 0),      # NMT head, padding id ignored
    (64, 1000, 1000, torch.float32, -100),
    (33, 136, 129, torch.bfloat16, -100),         # vector tail inside the valid columns
])
def test_xent_matches_fp32_reference(rows, ld, V, dtype, ignore):
    _native.hip()
    torch.manual_seed(0)
    x = (torch.randn(rows, ld, device=DEV) * 3).to(dtype).requires_grad_(True)
    y = torch.randint(0, V, (rows,), device=DEV)
    if ignore >= 0:
        y[::7] = ignore
    loss, correct, n = softmax_cross_entropy(x, y, V, ignore_index=ignore)
    assert loss.grad_fn is not None and type(loss.grad_fn).__name__.startswith("_XentFn")
    xr = x.detach().float().requires_grad_(True)
    lr, cr, nr = xent_ref(xr, y, V, ignore)
    torch.testing.assert_close(loss, lr, rtol=1e-5, atol=1e-5)
    assert int(correct) == int(cr) and int(n) == int(nr)
    (loss * 2.5).backward()
    (lr * 2.5).backward()
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=1e-6 if dtype == torch.bfloat16 else 1e-7)
    assert float(x.grad[:, V:].float().abs().max() if ld > V else 0.0) == 0.0


def test_xent_propagates_nan():
    _native.hip()
    x = torch.randn(8, 1024, device=DEV, dtype=torch.bfloat16)
    x[3, 17] = float("nan")
    y = torch.randint(0, 1024, (8,), device=DEV)
    loss, _, _ = softmax_cross_entropy(x, y)
    assert not torch.isfinite(loss)


def test_xent_argmax_first_maximum():
    _native.hip()
    x = torch.zeros(4, 256, device=DEV, dtype=torch.bfloat16)
    x[:, 5] = 2.0
    x[:, 200] = 2.0  # tie: the first maximum (5) is the prediction, as torch.argmax
    y = torch.tensor([5, 200, 5, 3], device=DEV)
    _, correct, _ = softmax_cross_entropy(x, y)
    assert int(correct) == 2


def test_split_dgrad_matches_reference():
    from vodascheduler_amd.ops import dense

    torch.manual_seed(0)
    dy = torch.randn(1280, 30528, device=DEV).to(torch.bfloat16)
    w = (torch.randn(30528, 768, device=DEV) * 0.02).to(torch.bfloat16)
    assert dense._split_count(1280, 30528, 768) > 1
    out = dense._dgrad(dy, w)
    ref = dy.float() @ w.float()
    assert out.dtype == torch.bfloat16 and out.shape == (1280, 768)
    err = float((out.float() - ref).norm() / ref.norm())
    assert err < 4e-3, err


def test_fused_embedding_flat_gradient_gpu():
    from vodascheduler_amd.models import cast_compute_weights_
    from vodascheduler_amd.ops.embedding import FusedEmbedding
    from vodascheduler_amd.ops.optim import FusedAdamW
    from vodascheduler_amd.utils.flat import grad_of

    torch.manual_seed(0)
    m = cast_compute_weights_(FusedEmbedding(30528, 768).to(DEV))
    opt = FusedAdamW(m.parameters(), lr=1e-4)
    opt.zero_grad()
    ids = torch.randint(0, 30522, (64, 128), device=DEV)
    dy = torch.randn(64, 128, 768, device=DEV).to(torch.bfloat16)
    m(ids).backward(dy)
    ref = torch.zeros(30528, 768, device=DEV).index_add_(0, ids.reshape(-1), dy.reshape(-1, 768).float())
    g = grad_of(m.weight)
    assert g.dtype == torch.float32
    torch.testing.assert_close(g, ref, rtol=1e-5, atol=1e-5)


def test_bert_head_loss_matches_stock_path():
    """BERT-base (2 layers) logits -> fused CE equals F.cross_entropy on the first vocab
    columns, and the padded vocab rows stay untouched by the loss gradient."""
    from vodascheduler_amd.models import WORKLOADS, prepare_model
    from vodascheduler_amd.models.transformer import BertBase

    torch.manual_seed(0)
    w = WORKLOADS["bert-base"]
    m = prepare_model(w, DEV)
    assert isinstance(m, BertBase) and m.mlm_out.weight.shape[0] == 30528 and m.num_classes == 30522
    b = w.make_batch(8, DEV, None)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss, correct, n = w.loss_metrics(m, b)
        logits = m(b[0], b[1], b[2])
    ref = F.cross_entropy(logits[:, :30522].float(), b[3].reshape(-1))
    torch.testing.assert_close(loss, ref, rtol=1e-4, atol=1e-4)
    assert int(n) == b[3].numel()


def test_xent_out_of_range_labels_excluded_from_mean():
    """rows whose label lies outside [0, V) get zero loss and gradient in the
    kernel, so they must not count toward the mean either (same predicate)."""
    _native.hip()
    torch.manual_seed(1)
    R, V = 96, 200
    x = torch.randn(R, V, device=DEV).requires_grad_(True)
    y = torch.randint(0, V, (R,), device=DEV)
    y[::5] = V + 3      # out of range
    y[1::11] = -7       # negative, not ignore_index
    loss, _, n = softmax_cross_entropy(x, y, V)
    ok = (y >= 0) & (y < V)
    assert int(n) == int(ok.sum())
    lr = F.cross_entropy(x.detach()[ok], y[ok])
    torch.testing.assert_close(loss, lr, rtol=1e-5, atol=1e-5)
