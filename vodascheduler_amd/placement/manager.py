"""Topology-aware placement with migration minimisation.

Reference: pkg/placement/placement_manager.go (``Place`` 306-332, ``releaseSlots`` 337-411,
``bestFit`` 415-487, ``bindNodes`` 492-522, ``score`` 534-544, ``updateJobStates`` 548-566,
``updatePodNodeName`` 571-617, ``constructStatusOnRestart`` 640-680).

Two levels, MI355X-first:
1. **Node level** (the reference algorithm): release slots of finished / shrunk jobs (the
   highest worker indices first), best-fit the requests onto empty *virtual* nodes with the
   real nodes' capacities, then bind virtual -> real nodes with Kuhn-Munkres maximising
   ``sum_job min(virtual.workers[job], real.workers[job])`` -- i.e. the number of workers
   that stay where they are.
2. **GPU-slot level** inside each node: the node's healthy GPUs form an xGMI full mesh
   (7 point-to-point links per GPU), so any k-subset is bandwidth-symmetric and disjoint jobs
   share no link.  What matters is keeping each worker on its GPU: a second Munkres binds the
   node's per-job slot demand to physical GPUs, maximising the workers that keep their GPU
   (drained GPUs simply vanish from the node's slot list and their workers migrate).

Fixes vs the reference: best-fit assigns the *remaining* request, not the
whole request, to the best-fit node (#4); a job's node order is deterministic (nodes it
already used first, in their old order), so worker indices do not shuffle between plans
(#5); virtual nodes only bind to real nodes of the same capacity.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field

from ..utils.metrics import PlacementMetrics
from .munkres import assign_max

Loc = tuple[str, int]  # (node name, GPU index)


@dataclass
class NodeState:
    name: str
    gpus: list[int]
    job_num_workers: dict[str, int] = field(default_factory=dict)

    @property
    def total_slots(self) -> int:
        return len(self.gpus)

    @property
    def free_slots(self) -> int:
        return self.total_slots - sum(self.job_num_workers.values())


@dataclass
class PlacementPlan:
    """Result of :meth:`PlacementManager.place`."""

    workers: dict[str, list[Loc]]                  # job -> worker index -> (node, gpu)
    migrated: dict[str, list[tuple[Loc, Loc]]]     # job -> [(old loc, new loc)]
    restarted: list[str]                           # jobs whose workers ALL moved ("launcher deleted")
    cross_node_jobs: int
    duration_s: float

    @property
    def num_migrated(self) -> int:
        return sum(len(v) for v in self.migrated.values())


class PlacementManager:
    """``naive=True``: the migration-naive baseline -- the same best-fit packing, but virtual
    nodes are bound to real nodes in index order and each node's GPUs are handed out in index
    order, ignoring where workers currently run (no Munkres at either level).  Used by the
    GPU-drain experiment to measure what the Munkres binding saves."""

    def __init__(self, scheduler_id: str, nodes: dict[str, list[int]] | None = None,
                 metrics: PlacementMetrics | None = None, naive: bool = False,
                 gpu_numa: dict[str, dict[int, int]] | None = None):
        """``gpu_numa``: node -> {GPU index: NUMA domain} from runtime topology discovery
        (utils/topology.py); a job's GPUs are then kept inside one NUMA domain when that costs
        no migration (tie-breaker)."""
        self.scheduler_id = scheduler_id
        self.naive = naive
        self.gpu_numa = {k: dict(v) for k, v in (gpu_numa or {}).items()}
        self.lock = threading.Lock()
        self.nodes: dict[str, NodeState] = {}
        self.job_nodes: dict[str, list[list]] = {}      # job -> ordered [[node, n], ...]
        self.worker_loc: dict[str, list[Loc]] = {}      # current worker locations
        self.metrics = metrics or PlacementMetrics(scheduler_id)
        for n, gpus in (nodes or {}).items():
            self.add_node(n, gpus)

    # ------------------------------ node events ------------------------------
    def add_node(self, name: str, gpus: list[int]) -> None:
        with self.lock:
            if name in self.nodes:
                self.nodes[name].gpus = sorted(gpus)
            else:
                self.nodes[name] = NodeState(name, sorted(gpus))

    def update_node(self, name: str, gpus: list[int]) -> None:
        """Capacity change (e.g. a drained GPU).  Workers on removed GPUs are re-placed at the
        next :meth:`place`."""
        self.add_node(name, gpus)

    def delete_node(self, name: str) -> None:
        with self.lock:
            self.nodes.pop(name, None)

    def drain_gpu(self, node: str, gpu: int) -> None:
        with self.lock:
            st = self.nodes[node]
            st.gpus = [g for g in st.gpus if g != gpu]

    def total_gpus(self) -> int:
        return sum(n.total_slots for n in self.nodes.values())

    # ------------------------------ main entry ------------------------------
    def place(self, job_requests: dict[str, int]) -> PlacementPlan:
        t0 = time.perf_counter()
        with self.lock:
            requests = {j: int(n) for j, n in job_requests.items() if n > 0}
            old_loc = {j: list(v) for j, v in self.worker_loc.items()}
            self._sync_node_counts_with_locations()
            self._release_slots(requests)
            virtual = [NodeState(f"virtual-{i}", list(n.gpus)) for i, n in enumerate(self._node_list())]
            cross = self._best_fit(requests, virtual)
            self._bind_nodes(virtual)
            self._update_job_states()
            plan = self._bind_gpus(old_loc)
        plan.cross_node_jobs = cross
        plan.duration_s = time.perf_counter() - t0
        self.metrics.algo_duration.observe(plan.duration_s)
        self.metrics.workers_migrated.set(plan.num_migrated)
        self.metrics.launchers_deleted.set(len(plan.restarted))
        self.metrics.jobs_cross_node.set(cross)
        return plan

    # ------------------------------ steps ------------------------------
    def _node_list(self) -> list[NodeState]:
        return [self.nodes[k] for k in sorted(self.nodes)]

    def _sync_node_counts_with_locations(self) -> None:
        """Rebuild node job counts from the worker locations (drops GPUs that vanished)."""
        for n in self.nodes.values():
            n.job_num_workers = {}
        new_job_nodes: dict[str, list[list]] = {}
        for job, locs in self.worker_loc.items():
            order: list[list] = []
            for node, gpu in locs:
                st = self.nodes.get(node)
                if st is None or gpu not in st.gpus:
                    continue  # node deleted / GPU drained: that worker must move
                st.job_num_workers[job] = st.job_num_workers.get(job, 0) + 1
                for e in order:
                    if e[0] == node:
                        e[1] += 1
                        break
                else:
                    order.append([node, 1])
            if order:
                new_job_nodes[job] = order
        self.job_nodes = new_job_nodes

    def _release_slots(self, requests: dict[str, int]) -> None:
        for job, order in list(self.job_nodes.items()):
            want = requests.get(job, 0)
            have = sum(n for _, n in order)
            if want == 0:
                for node, n in order:
                    if node in self.nodes:
                        self.nodes[node].job_num_workers.pop(job, None)
                self.job_nodes.pop(job)
                continue
            to_release = have - want
            while to_release > 0 and order:  # highest worker indices = last nodes first
                node, n = order[-1]
                st = self.nodes.get(node)
                r = min(n, to_release)
                order[-1][1] -= r
                to_release -= r
                if st is not None:
                    st.job_num_workers[job] -= r
                    if st.job_num_workers[job] == 0:
                        del st.job_num_workers[job]
                if order[-1][1] == 0:
                    order.pop()

    @staticmethod
    def _best_fit(requests: dict[str, int], nodes: list[NodeState]) -> int:
        """Best-fit bin packing of job requests onto (empty) nodes; returns #cross-node jobs."""
        reqs = sorted(requests.items(), key=lambda kv: (-kv[1], kv[0]))
        total_slots = sum(n.total_slots for n in nodes)
        cross_jobs = set()
        for job, n in reqs:
            requested = n
            while requested > 0:
                if total_slots == 0:
                    return len(cross_jobs)  # tolerate scheduler/placement inconsistency
                best, mx = -1, 0
                for i, node in enumerate(nodes):
                    if node.free_slots >= requested and (best == -1 or nodes[best].free_slots > node.free_slots):
                        best = i
                    if nodes[mx].free_slots < node.free_slots:
                        mx = i
                if best == -1:
                    take = nodes[mx].free_slots
                    if take == 0:
                        return len(cross_jobs)
                    nodes[mx].job_num_workers[job] = nodes[mx].job_num_workers.get(job, 0) + take
                    requested -= take
                    total_slots -= take
                    cross_jobs.add(job)
                else:
                    nodes[best].job_num_workers[job] = nodes[best].job_num_workers.get(job, 0) + requested
                    total_slots -= requested
                    requested = 0
        return len(cross_jobs)

    def _bind_nodes(self, virtual: list[NodeState]) -> None:
        real = self._node_list()
        if not real:
            return
        size = len(real)
        if self.naive:
            for vi, v in enumerate(virtual[:size]):
                real[vi].job_num_workers = dict(v.job_num_workers)
            return
        big = 10 ** 6
        scores = []
        for v in virtual:
            row = []
            for r in real:
                if v.total_slots != r.total_slots:
                    row.append(-big)
                    continue
                row.append(sum(min(w, r.job_num_workers.get(j, 0)) for j, w in v.job_num_workers.items()))
            scores.append(row)
        assign = assign_max(scores)
        for vi, ri in enumerate(assign):
            if ri < 0 or ri >= size:
                continue
            real[ri].job_num_workers = dict(virtual[vi].job_num_workers)

    def _update_job_states(self) -> None:
        new: dict[str, list[list]] = {}
        for node in self._node_list():
            for job, w in node.job_num_workers.items():
                if w > 0:
                    new.setdefault(job, []).append([node.name, w])
        for job, lst in new.items():
            prev = [n for n, _ in self.job_nodes.get(job, [])]
            lst.sort(key=lambda e: (prev.index(e[0]) if e[0] in prev else len(prev), e[0]))
        self.job_nodes = new

    def _bind_gpus(self, old_loc: dict[str, list[Loc]]) -> PlacementPlan:
        """Per node: Munkres from per-job slot demand to physical GPUs, keeping workers put."""
        gpu_of: dict[str, dict[str, list[int]]] = {}  # node -> job -> gpus
        for node in self._node_list():
            slots: list[str] = []
            for job in sorted(node.job_num_workers):
                slots += [job] * node.job_num_workers[job]
            occupant: dict[int, tuple[str, int]] = {}
            for job, locs in old_loc.items():
                for idx, (n, g) in enumerate(locs):
                    if n == node.name and g in node.gpus:
                        occupant[g] = (job, idx)
            gpus = node.gpus
            if not slots:
                gpu_of[node.name] = {}
                continue
            # keeping a worker on its GPU scores 2 (+ up to 0.5 for low old worker indices, so a
            # shrinking job keeps its lowest ranks -- rank 0 holds the state); a GPU in the job's
            # preferred NUMA domain scores 0.1 (never outweighs a kept worker); tie-break to
            # lower GPU ids
            numa = self.gpu_numa.get(node.name, {})
            pref = self._preferred_numa(node, numa, occupant) if numa and not self.naive else {}
            buddy = self._buddy_blocks(node, occupant) if not self.naive else {}

            def score(job: str, k: int, g: int) -> float:
                occ = occupant.get(g)
                s = 0.0
                if occ is not None and occ[0] == job and not self.naive:
                    s = 2.0 + 0.5 / (1 + occ[1])
                if job in pref and numa.get(g) == pref[job]:
                    s += 0.1
                if g in buddy.get(job, ()):
                    s += 0.05
                return s - 1e-6 * k

            scores = [[score(job, k, g) for k, g in enumerate(gpus)] for job in slots]
            assign = assign_max(scores)
            m: dict[str, list[int]] = {}
            for job, gi in zip(slots, assign):
                m.setdefault(job, []).append(gpus[gi])
            gpu_of[node.name] = m
        workers: dict[str, list[Loc]] = {}
        migrated: dict[str, list[tuple[Loc, Loc]]] = {}
        restarted: list[str] = []
        for job, order in self.job_nodes.items():
            new_set: list[Loc] = []
            for node, _n in order:
                new_set += [(node, g) for g in sorted(gpu_of[node].get(job, []))]
            old = old_loc.get(job, [])
            kept = [l for l in old if l in new_set]
            fresh = [l for l in new_set if l not in kept]
            workers[job] = kept + fresh  # surviving workers keep their ranks (rank 0 survives)
            gone = [l for l in old if l not in new_set]
            moves = min(len(old), len(new_set)) - len(kept)
            if moves > 0:
                migrated[job] = list(zip(gone[:moves], fresh[:moves]))
            if old and new_set and not kept:
                restarted.append(job)
        self.worker_loc = workers
        return PlacementPlan(workers=workers, migrated=migrated, restarted=restarted, cross_node_jobs=0,
                             duration_s=0.0)

    @staticmethod
    def _buddy_blocks(node: NodeState, occupant: dict[int, tuple[str, int]]) -> dict[str, set[int]]:
        """Per job on this node: an aligned block of next_pow2(demand) GPU positions (buddy
        allocation: [0,1], [2,3], [0..3], ...) it should fill.  A job that already holds GPUs
        here prefers the block around them (it grows into its buddy); new arrivals, largest
        demand first, take the lowest wholly free block.  Aligned sets recur across jobs and
        resizes, so their RCCL communicators come out of the per-worker communicator cache
        (pre-built for every aligned group by bench.py's warm-up) instead of a new bootstrap;
        they also keep the free GPUs unfragmented.  A preference only: kept workers (2.0) and
        the NUMA domain (0.1) weigh more."""
        gpus = node.gpus
        n = len(gpus)
        pos = {g: i for i, g in enumerate(gpus)}
        taken: set[int] = {pos[g] for g in occupant if g in pos}
        out: dict[str, set[int]] = {}
        have: dict[str, list[int]] = {}
        for g, (j, _i) in occupant.items():
            if g in pos:
                have.setdefault(j, []).append(pos[g])
        order = sorted(node.job_num_workers, key=lambda j: (j not in have, -node.job_num_workers[j], j))
        claimed: set[int] = set()
        for job in order:
            d = node.job_num_workers[job]
            size = 1
            while size < d:
                size *= 2
            if size > n:
                continue
            mine = set(have.get(job, []))
            best = None
            for b0 in range(0, n - size + 1, size):
                block = set(range(b0, b0 + size))
                foreign = (block & taken) - mine
                if foreign or (block & claimed):
                    continue
                key = (-len(block & mine), b0)  # most of my GPUs first, then the lowest block
                if best is None or key < best[0]:
                    best = (key, block)
            if best is None:
                continue
            claimed |= best[1]
            out[job] = {gpus[i] for i in best[1]}
        return out

    @staticmethod
    def _preferred_numa(node: NodeState, numa: dict[int, int], occupant: dict[int, tuple[str, int]]) -> dict[str, int]:
        """Per job on this node: the NUMA domain holding most of its current workers, else
        (new arrivals, largest demand first) the domain with the most GPUs left unclaimed."""
        free: dict[int, int] = {}
        for g in node.gpus:
            if g not in occupant:
                free[numa.get(g, 0)] = free.get(numa.get(g, 0), 0) + 1
        pref: dict[str, int] = {}
        for job in sorted(node.job_num_workers, key=lambda j: (-node.job_num_workers[j], j)):
            have: dict[int, int] = {}
            for g, (oj, _i) in occupant.items():
                if oj == job and g in node.gpus:
                    have[numa.get(g, 0)] = have.get(numa.get(g, 0), 0) + 1
            if have:
                pref[job] = max(have, key=lambda d: (have[d], -d))
            elif free:
                d = max(free, key=lambda x: (free[x], -x))
                pref[job] = d
                free[d] -= min(free[d], node.job_num_workers[job])
        return pref

    # ------------------------------ restart ------------------------------
    def construct_status_on_restart(self, worker_loc: dict[str, list[Loc]]) -> None:
        """Rebuild node/job state from observed worker locations (reference recovers them
        from pod tolerations, placement_manager.go:640-680)."""
        with self.lock:
            self.worker_loc = {j: list(v) for j, v in worker_loc.items()}
            self._sync_node_counts_with_locations()
