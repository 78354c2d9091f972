"""Runtime discovery of a node's GPU interconnect and NUMA layout.

Source: the KFD topology in sysfs (``/sys/class/kfd/kfd/topology/nodes/<n>/properties`` and
``.../io_links/<k>/properties``), which lists every CPU and GPU agent of the machine and
every link between them with its type and weight: ``type 11`` = xGMI, ``type 2`` = PCIe
(GPU <-> CPU socket), ``type 1`` = CPU <-> CPU.  On an 8 x MI355X node each GPU has 7 xGMI
links (weight 15, one per peer: a full mesh) and one PCIe link to its NUMA node's CPU
(tests/fixtures/mi355x_kfd_topology_1gpu_box.txt was captured on one such box; inside a
1-GPU container the peers' own property files are not readable, so the mesh is
reconstructed from the links that are).

GPU index = rank of the GPU agent among the GPU agents in KFD node order, which is the order
ROCr (and therefore HIP / ``torch.cuda``) enumerates devices in.

Consumers:
* placement (``placement/manager.py``): tie-break GPU choice toward one NUMA domain / one
  xGMI clique;
* bucket sizing (``bucket_cap_mb``): per-step chunk = bucket / (channels x k), channels ~ links;
* NUMA affinity of pool workers (``numa_cpus`` -> ``os.sched_setaffinity``).
"""
from __future__ import annotations

import glob
import os
import re
from dataclasses import dataclass, field

KFD_ROOT = "/sys/class/kfd/kfd/topology/nodes"
LINK_XGMI, LINK_PCIE, LINK_CPU = 11, 2, 1


@dataclass
class Topology:
    gpus: list[int]                                  # KFD node ids of the GPUs, in device order
    numa: dict[int, int] = field(default_factory=dict)          # GPU index -> NUMA node (CPU agent order)
    xgmi: dict[tuple[int, int], int] = field(default_factory=dict)  # (i, j) GPU indices -> link weight
    xgmi_bw_mbs: dict[tuple[int, int], int] = field(default_factory=dict)
    source: str = ""

    @property
    def n(self) -> int:
        return len(self.gpus)

    def links_per_gpu(self) -> int:
        if not self.gpus:
            return 0
        return max(sum(1 for (a, _b) in self.xgmi if a == i) for i in range(self.n))

    def full_mesh(self) -> bool:
        """Every GPU pair is one xGMI hop (any k-subset is bandwidth-symmetric)."""
        return self.n > 0 and all((i, j) in self.xgmi for i in range(self.n) for j in range(self.n) if i != j)

    def numa_groups(self) -> dict[int, list[int]]:
        out: dict[int, list[int]] = {}
        for g in range(self.n):
            out.setdefault(self.numa.get(g, 0), []).append(g)
        return out

    def bucket_mb(self, k: int, step_latency_us: float = 5.0, link_gbs: float | None = None) -> float:
        """All-reduce bucket that amortises the per-step ring latency on ``k`` GPUs:
        bucket >~ alpha * beta * channels * k, rounded up to a power of two
        in [32, 256] MB."""
        if link_gbs is None:
            bws = list(self.xgmi_bw_mbs.values())
            link_gbs = (max(bws) / 1000.0) if bws else 64.0
        ch = max(1, self.links_per_gpu())
        need = step_latency_us * 1e-6 * link_gbs * 1e9 * ch * max(1, k) / 2 ** 20
        mb = 32
        while mb < need and mb < 256:
            mb *= 2
        return float(mb)


def _read_props(path: str) -> dict[str, int]:
    out: dict[str, int] = {}
    try:
        with open(path) as f:
            for line in f:
                p = line.split()
                if len(p) == 2:
                    try:
                        out[p[0]] = int(p[1])
                    except ValueError:
                        pass
    except OSError:
        pass
    return out


def _parse_dump(text: str) -> tuple[dict[int, dict], list[dict]]:
    """Parse a ``== <path>`` / ``key value`` dump of the sysfs files (the fixture format)."""
    nodes: dict[int, dict] = {}
    links: list[dict] = []
    for block in re.split(r"^== ", text, flags=re.M)[1:]:
        head, *lines = block.strip().split("\n")
        kv: dict[str, int] = {}
        for line in lines:
            p = line.split()
            if len(p) == 2:
                try:
                    kv[p[0]] = int(p[1])
                except ValueError:
                    pass
        m = re.search(r"nodes/(\d+)/io_links/(\d+)/properties", head)
        if m:
            if kv:
                kv.setdefault("node_from", int(m.group(1)))
                links.append(kv)
            continue
        m = re.search(r"nodes/(\d+)/properties", head)
        if m:
            nodes[int(m.group(1))] = kv
    return nodes, links


def _read_sysfs(root: str) -> tuple[dict[int, dict], list[dict]]:
    nodes: dict[int, dict] = {}
    links: list[dict] = []
    for d in sorted(glob.glob(os.path.join(root, "*")), key=lambda p: int(os.path.basename(p)) if
                    os.path.basename(p).isdigit() else -1):
        name = os.path.basename(d)
        if not name.isdigit():
            continue
        nid = int(name)
        nodes[nid] = _read_props(os.path.join(d, "properties"))
        for lp in sorted(glob.glob(os.path.join(d, "io_links", "*", "properties"))):
            kv = _read_props(lp)
            if kv:
                kv.setdefault("node_from", nid)
                links.append(kv)
    return nodes, links


def build(nodes: dict[int, dict], links: list[dict], source: str = "") -> Topology:
    cpu_nodes = {n for n, kv in nodes.items() if kv.get("cpu_cores_count", 0) > 0 and kv.get("simd_count", 0) == 0}
    gpu_nodes = {n for n, kv in nodes.items() if kv.get("simd_count", 0) > 0}
    for l in links:  # agents whose own properties are unreadable still show up as link ends
        if l.get("type") == LINK_XGMI:
            gpu_nodes.update((l["node_from"], l["node_to"]))
        elif l.get("type") == LINK_PCIE:
            a, b = l["node_from"], l["node_to"]
            if a in cpu_nodes:
                gpu_nodes.add(b)
            elif b in cpu_nodes:
                gpu_nodes.add(a)
    gpu_nodes -= cpu_nodes
    order = sorted(gpu_nodes)
    idx = {n: i for i, n in enumerate(order)}
    cpu_order = {n: i for i, n in enumerate(sorted(cpu_nodes))}
    t = Topology(gpus=order, source=source)
    for l in links:
        a, b, ty = l.get("node_from"), l.get("node_to"), l.get("type")
        if ty == LINK_XGMI and a in idx and b in idx:
            for x, y in ((a, b), (b, a)):  # links are symmetric; a 1-GPU container sees one side
                t.xgmi.setdefault((idx[x], idx[y]), int(l.get("weight", 0)))
                bw = int(l.get("max_bandwidth", 0))
                if bw:
                    t.xgmi_bw_mbs.setdefault((idx[x], idx[y]), bw)
        elif ty == LINK_PCIE:
            if a in idx and b in cpu_order:
                t.numa[idx[a]] = cpu_order[b]
            elif b in idx and a in cpu_order:
                t.numa[idx[b]] = cpu_order[a]
    # the peers' xGMI links to each other are not visible from a 1-GPU container: a GPU that
    # reaches every other GPU directly implies the vendor's all-to-all mesh (MI355X UBB)
    if order and any(sum(1 for (x, _y) in t.xgmi if x == i) == len(order) - 1 for i in range(len(order))):
        w = max(t.xgmi.values())
        bw = max(t.xgmi_bw_mbs.values()) if t.xgmi_bw_mbs else 0
        for i in range(len(order)):
            for j in range(len(order)):
                if i != j:
                    t.xgmi.setdefault((i, j), w)
                    if bw:
                        t.xgmi_bw_mbs.setdefault((i, j), bw)
    return t


def discover(root: str = KFD_ROOT) -> Topology:
    """Topology of this machine from sysfs (empty Topology when KFD is absent, e.g. CPU-only)."""
    if not os.path.isdir(root):
        return Topology(gpus=[], source="none")
    nodes, links = _read_sysfs(root)
    return build(nodes, links, source=root)


def from_dump(text: str) -> Topology:
    nodes, links = _parse_dump(text)
    return build(nodes, links, source="dump")


def gpu_local_cpus(device_index: int) -> list[int]:
    """CPUs local to HIP device ``device_index`` (its PCI device's ``local_cpulist``),
    intersected with this process's allowed CPUs.  [] if unknown."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device_index)
        bdf = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    except Exception:
        return []
    path = f"/sys/bus/pci/devices/{bdf}/local_cpulist"
    try:
        with open(path) as f:
            cpus = parse_cpulist(f.read())
    except OSError:
        return []
    allowed = os.sched_getaffinity(0)
    return sorted(c for c in cpus if c in allowed)


def parse_cpulist(s: str) -> list[int]:
    out: list[int] = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def pin_to_gpu_numa(device_index: int) -> list[int]:
    """Pin the calling process to the CPUs local to its GPU (NUMA affinity of a pool worker:
    host-side batch staging and kernel launches stay on the GPU's socket).  Returns the CPU
    set applied ([] = left unchanged)."""
    cpus = gpu_local_cpus(device_index)
    if cpus:
        try:
            os.sched_setaffinity(0, cpus)
        except OSError:
            return []
    return cpus
