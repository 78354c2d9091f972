"""Adasum reduction (Horovod op=hvd.Adasum, reference pytorch_mnist_elastic.py:32,188):
algebraic properties of the reference, the DDP engine over gloo with 2 and 3 ranks on CPU,
and the HIP segmented combine kernels against the fp32 reference on the GPU."""
import multiprocessing as mp

import pytest
import torch

from vodascheduler_amd.ops.adasum import AdasumPlan, adasum_pair_, adasum_pair_ref, adasum_tree_, adasum_tree_ref
from vodascheduler_amd.parallel.comm import GlooCommunicator
from vodascheduler_amd.parallel.ddp import ElasticDDP
from vodascheduler_amd.runtime.cluster import free_port
from vodascheduler_amd.runtime.rendezvous import connect_store


def test_adasum_identical_is_identity_and_orthogonal_is_sum():
    a = torch.randn(100)
    torch.testing.assert_close(adasum_pair_ref(a, a, [(0, 100)]), a)
    b = torch.zeros(100)
    b[:50] = torch.randn(50)
    a2 = torch.zeros(100)
    a2[50:] = torch.randn(50)
    torch.testing.assert_close(adasum_pair_ref(a2, b, [(0, 100)]), a2 + b)
    # zero operand: adasum(a, 0) == a
    torch.testing.assert_close(adasum_pair_ref(a, torch.zeros(100), [(0, 100)]), a)


def test_adasum_is_per_segment():
    a, b = torch.randn(64), torch.randn(64)
    segs = [(0, 10), (10, 64)]
    out = adasum_pair_ref(a, b, segs)
    torch.testing.assert_close(out[:10], adasum_pair_ref(a[:10], b[:10], [(0, 10)]))
    torch.testing.assert_close(out[10:], adasum_pair_ref(a[10:], b[10:], [(0, 54)]))


def test_adasum_plan_validates_tiling():
    with pytest.raises(ValueError):
        AdasumPlan([(0, 10), (12, 20)], torch.device("cpu"))
    p = AdasumPlan([(0, 40000), (40000, 40001)], torch.device("cpu"), chunk=16384)
    assert p.nseg == 2 and p.nblk == 3 + 1 and p.numel == 40001


def test_adasum_tree_cpu_matches_ref_non_power_of_two():
    rows = torch.randn(5, 300)
    segs = [(0, 100), (100, 300)]
    plan = AdasumPlan(segs, torch.device("cpu"))
    ref = adasum_tree_ref(list(rows), segs)
    out = adasum_tree_(rows.clone(), plan)
    torch.testing.assert_close(out, ref)


def _adasum_worker(port, rank, world, q):
    torch.set_num_threads(1)
    store = connect_store("127.0.0.1", port)
    comm = GlooCommunicator(store, "t/adasum", rank, world, timeout=60)
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(16, 300), torch.nn.ReLU(), torch.nn.Linear(300, 4))
    ddp = ElasticDDP(m, comm, None, bucket_cap_mb=0.001, first_bucket_mb=0.0005, reduction="adasum")
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(8, 16, generator=g)
    ddp.zero_grad()
    m(x).square().mean().backward()
    ddp.finalize()
    q.put((rank, [p.grad.numpy().copy() for p in m.parameters()], x.numpy().copy()))


@pytest.mark.parametrize("world", [2, 3])
def test_ddp_adasum_matches_per_tensor_reference(world):
    port = free_port()
    store = connect_store("127.0.0.1", port, is_master=True)  # noqa: F841
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_adasum_worker, args=(port, r, world, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r, ([torch.from_numpy(a) for a in g], torch.from_numpy(x)))
               for r, g, x in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(30)
    # per-rank local gradients, combined per parameter tensor along the same tree
    local = []
    for r in range(world):
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(16, 300), torch.nn.ReLU(), torch.nn.Linear(300, 4))
        m(res[r][1]).square().mean().backward()
        local.append([p.grad.clone() for p in m.parameters()])
    for i in range(len(local[0])):
        rows = [local[r][i].reshape(-1) for r in range(world)]
        ref = adasum_tree_ref(rows, [(0, rows[0].numel())]).view_as(local[0][i])
        for r in range(world):
            torch.testing.assert_close(res[r][0][i], ref, rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(res[0][0][i], res[world - 1][0][i], rtol=0, atol=0)  # replicas agree bitwise


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_adasum_pair_kernel_matches_ref(dtype):
    dev = torch.device("cuda", 0)
    # segments: tiny, unaligned boundaries, one spanning several 16K-element chunks
    bounds = [0, 3, 67, 64 * 5, 40000, 40001, 100032]
    segs = list(zip(bounds[:-1], bounds[1:]))
    n = bounds[-1]
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn(n, device=dev, generator=g).to(dtype)
    b = (0.5 * a.float() + torch.randn(n, device=dev, generator=g)).to(dtype)
    plan = AdasumPlan(segs, dev)
    out = torch.empty_like(a)
    adasum_pair_(a, b, out, plan)
    ref = adasum_pair_ref(a.cpu(), b.cpu(), segs)
    tol = dict(rtol=1e-5, atol=1e-5) if dtype == torch.float32 else dict(rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(out.float().cpu(), ref, **tol)
    # in place (out aliases a) and deterministic
    a2 = a.clone()
    adasum_pair_(a2, b, a2, plan)
    torch.testing.assert_close(a2, out, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_adasum_tree_kernel_matches_ref(world):
    dev = torch.device("cuda", 0)
    segs = [(0, 4096), (4096, 4160), (4160, 300000)]
    rows = torch.randn(world, 300000, device=dev)
    plan = AdasumPlan(segs, dev)
    out = adasum_tree_(rows.clone(), plan).cpu()
    ref = adasum_tree_ref(list(rows.cpu()), segs)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-5)
