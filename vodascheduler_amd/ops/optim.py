"""Fused flat-buffer optimizers: SGD(+momentum/nesterov), Adam/AdamW, RMSprop.

GPU path: ONE HIP launch per parameter group per step (csrc/hip/optim.hip), reading
param/grad/state once, optionally writing the bf16/fp16 model-weight copy in the same
pass.  CPU path: the same math in PyTorch ops on the same flat buffers (reference used
by the numerics tests).  Semantics follow ``torch.optim`` so the reference workloads'
optimizers (SGD momentum 0.9 for ResNet50/VGG16, Adam for MNIST, RMSprop for
InceptionV3/Transformer — reference examples/yaml/tensorflow2/*.yaml and SURVEY.md §2.8)
map one-to-one.
"""
from __future__ import annotations

import math

import torch

from ..utils.flat import FlatGroup
from . import _native as N


def _split_by_dtype(params) -> list[dict]:
    """Param groups with one dtype each: a model whose GEMM/conv weights are stored in bf16
    (``models.cast_compute_weights_``) and whose norm parameters stay fp32 gets one flat
    group per dtype -- the bf16 group keeps an fp32 master + bf16 model copy + bf16 grads."""
    params = list(params)
    groups = params if params and isinstance(params[0], dict) else [{"params": params}]
    out = []
    for g in groups:
        ps = list(g["params"])
        by: dict[torch.dtype, list] = {}
        for p in ps:
            by.setdefault(p.dtype, []).append(p)
        for dt in sorted(by, key=str):
            out.append({**g, "params": by[dt]})
    return out


class _FusedFlatOptimizer(torch.optim.Optimizer):
    """Base class: owns one :class:`FlatGroup` per param group."""

    _state_names: tuple[str, ...] = ()

    def __init__(self, params, defaults, grad_dtype: torch.dtype | None = None):
        super().__init__(_split_by_dtype(params), defaults)
        self.flat_groups: list[FlatGroup] = []
        self._flat_state: list[dict[str, torch.Tensor]] = []
        self._steps: list[int] = []
        for g in self.param_groups:
            # a low-precision gradient request applies to low-precision (bf16/fp16) weights only;
            # fp32 parameters (norm layers) always keep fp32 gradients
            pdt = g["params"][0].dtype if g["params"] else torch.float32
            gdt = grad_dtype if (grad_dtype is not None and pdt != torch.float32) else torch.float32
            fg = FlatGroup(g["params"], flatten_params=True, grad_dtype=gdt)
            self.flat_groups.append(fg)
            self._flat_state.append({})
            self._steps.append(0)
        # Per-group step counters on the device.  They are part of the synced/checkpointed
        # state (a rank that joins a running job must use the same Adam bias correction as
        # the others) and are what the kernels read, so a step captured in a hipGraph stays
        # correct on every replay.
        self._step_t = torch.zeros(len(self.param_groups), dtype=torch.int64, device=self.flat_groups[0].device)

    # -- state buffers (allocated lazily, flat fp32) --
    def _buf(self, gi: int, name: str) -> torch.Tensor:
        st = self._flat_state[gi]
        if name not in st:
            st[name] = torch.zeros_like(self.flat_groups[gi].master)
        return st[name]

    def zero_grad(self, set_to_none: bool = False) -> None:  # grads are flat views: never None
        for fg in self.flat_groups:
            fg.zero_grad()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self.begin_step()
        for gi, fg in enumerate(self.flat_groups):
            self.step_range(gi, 0, fg.numel)
        return loss

    @torch.no_grad()
    def begin_step(self) -> None:
        """Advance the step counters (host + device) once per training step; the updates then
        run as one ``step_range`` per group or per gradient bucket (parallel/ddp.py overlaps
        them with backward)."""
        self._step_t.add_(1)
        for gi in range(len(self._steps)):
            self._steps[gi] += 1

    @torch.no_grad()
    def step_range(self, gi: int, start: int, end: int) -> None:
        """Update flat elements ``[start, end)`` of group ``gi`` (bucket boundaries are slot
        offsets: 64-element aligned, so every sliced pointer stays 256-byte aligned)."""
        if end <= start:
            return
        group, fg = self.param_groups[gi], self.flat_groups[gi]
        if fg.master.is_cuda:
            self._step_gpu(gi, group, fg, start, end)
        else:
            self._step_cpu(gi, group, fg, start, end)

    def _lowp_args(self, fg: FlatGroup, start: int = 0) -> tuple[int, int]:
        if fg.lowp is None:
            return 0, -1
        return fg.lowp.data_ptr() + start * fg.lowp.element_size(), N.dtype_code(fg.lowp.dtype)

    @staticmethod
    def _at(t: torch.Tensor | None, start: int) -> int:
        """Device pointer of element ``start`` of a flat buffer (0 for None)."""
        return 0 if t is None else t.data_ptr() + start * t.element_size()

    def _check(self, fg: FlatGroup) -> None:
        N.check_gpu_tensor(fg.master, "master")
        N.check_gpu_tensor(fg.grad, "grad", align=8)
        if fg.grad.numel() != fg.master.numel():
            raise ValueError("grad/master size mismatch")

    # -- checkpoint / elastic state sync --
    def flat_state_tensors(self) -> list[torch.Tensor]:
        """All tensors that define the optimizer+model state (for broadcast/snapshot)."""
        out = []
        for gi, fg in enumerate(self.flat_groups):
            out.append(fg.master)
            for name in self._state_names_for(gi):
                out.append(self._buf(gi, name))
        out.append(self._step_t)
        return out

    def reset_steps(self) -> None:
        self._steps = [0] * len(self._steps)
        self._step_t.zero_()

    def advance_host_steps(self, n: int = 1) -> None:
        """Host mirror of the device counters after ``n`` replays of a captured step."""
        self._steps = [s + n for s in self._steps]

    def _state_names_for(self, gi: int) -> tuple[str, ...]:
        return self._state_names

    def state_dict(self):
        sd = {"param_groups": [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups],
              "steps": list(self._steps), "flat": []}
        for gi, fg in enumerate(self.flat_groups):
            d = {"master": fg.master}
            for name in self._state_names_for(gi):
                d[name] = self._buf(gi, name)
            sd["flat"].append(d)
        return sd

    @torch.no_grad()
    def load_state_dict(self, sd):
        if len(sd["flat"]) != len(self.flat_groups):
            raise ValueError("param group count mismatch")
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            g.update(sg)
        self._steps = list(sd["steps"])
        self._step_t.copy_(torch.tensor(self._steps, dtype=torch.int64))
        for gi, (fg, d) in enumerate(zip(self.flat_groups, sd["flat"])):
            fg.master.copy_(d["master"])
            for name in self._state_names_for(gi):
                if name in d:
                    self._buf(gi, name).copy_(d[name])
            fg.sync_lowp_from_master()

    def after_external_update(self) -> None:
        """Call after master buffers / step counters were overwritten (broadcast/restore)."""
        for fg in self.flat_groups:
            fg.sync_lowp_from_master()
        self._steps = [int(x) for x in self._step_t.tolist()]


class FusedSGD(_FusedFlatOptimizer):
    def __init__(self, params, lr: float, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, grad_scale: float = 1.0,
                 grad_dtype: torch.dtype | None = None):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening,
                                      weight_decay=weight_decay, nesterov=nesterov, grad_scale=grad_scale),
                         grad_dtype)

    def _state_names_for(self, gi):
        return ("momentum_buffer",) if self.param_groups[gi]["momentum"] != 0 else ()

    def _step_gpu(self, gi, g, fg, start=0, end=None):
        end = fg.numel if end is None else end
        self._check(fg)
        mom = g["momentum"]
        buf = self._buf(gi, "momentum_buffer") if mom != 0 else None
        lp, lpdt = self._lowp_args(fg, start)
        N.hip().sgd_step(self._at(fg.master, start), self._at(fg.grad, start), N.dtype_code(fg.grad.dtype),
                         self._at(buf, start), lp, lpdt, end - start, float(g["lr"]), float(mom),
                         float(g["dampening"]), float(g["weight_decay"]), bool(g["nesterov"]), self._steps[gi] == 1,
                         float(g["grad_scale"]), N.stream_of(fg.master))

    def _step_cpu(self, gi, g, fg, start=0, end=None):
        sl = slice(start, fg.numel if end is None else end)
        p = fg.master[sl]
        d = fg.grad[sl].float() * g["grad_scale"]
        if g["weight_decay"] != 0:
            d = d + g["weight_decay"] * p
        if g["momentum"] != 0:
            buf = self._buf(gi, "momentum_buffer")[sl]
            if self._steps[gi] == 1:
                buf.copy_(d)
            else:
                buf.mul_(g["momentum"]).add_(d, alpha=1 - g["dampening"])
            d = d + g["momentum"] * buf if g["nesterov"] else buf
        p.add_(d, alpha=-g["lr"])
        _sync_lowp(fg, sl)


class FusedAdam(_FusedFlatOptimizer):
    _state_names = ("exp_avg", "exp_avg_sq")

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, adamw: bool = False, grad_scale: float = 1.0,
                 grad_dtype: torch.dtype | None = None):
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                                      adamw=adamw, grad_scale=grad_scale), grad_dtype)

    def _step_gpu(self, gi, g, fg, start=0, end=None):
        end = fg.numel if end is None else end
        self._check(fg)
        m, v = self._buf(gi, "exp_avg"), self._buf(gi, "exp_avg_sq")
        lp, lpdt = self._lowp_args(fg, start)
        b1, b2 = g["betas"]
        N.hip().adam_step(self._at(fg.master, start), self._at(fg.grad, start), N.dtype_code(fg.grad.dtype),
                          self._at(m, start), self._at(v, start), lp, lpdt, end - start, float(g["lr"]), float(b1),
                          float(b2), float(g["eps"]), float(g["weight_decay"]), bool(g["adamw"]), self._steps[gi],
                          float(g["grad_scale"]), self._step_t.data_ptr() + gi * 8, N.stream_of(fg.master))

    def _step_cpu(self, gi, g, fg, start=0, end=None):
        sl = slice(start, fg.numel if end is None else end)
        p = fg.master[sl]
        m, v = self._buf(gi, "exp_avg")[sl], self._buf(gi, "exp_avg_sq")[sl]
        b1, b2 = g["betas"]
        t = self._steps[gi]
        d = fg.grad[sl].float() * g["grad_scale"]
        if g["adamw"]:
            p.mul_(1 - g["lr"] * g["weight_decay"])
        elif g["weight_decay"] != 0:
            d = d + g["weight_decay"] * p
        m.mul_(b1).add_(d, alpha=1 - b1)
        v.mul_(b2).addcmul_(d, d, value=1 - b2)
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        denom = (v.sqrt() / math.sqrt(bc2)).add_(g["eps"])
        p.addcdiv_(m, denom, value=-g["lr"] / bc1)
        _sync_lowp(fg, sl)


class FusedAdamW(FusedAdam):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, grad_scale: float = 1.0, grad_dtype: torch.dtype | None = None):
        super().__init__(params, lr, betas, eps, weight_decay, adamw=True, grad_scale=grad_scale,
                         grad_dtype=grad_dtype)


class FusedRMSprop(_FusedFlatOptimizer):
    def __init__(self, params, lr: float = 1e-2, alpha: float = 0.99, eps: float = 1e-8,
                 weight_decay: float = 0.0, momentum: float = 0.0, centered: bool = False,
                 grad_scale: float = 1.0, grad_dtype: torch.dtype | None = None):
        super().__init__(params, dict(lr=lr, alpha=alpha, eps=eps, weight_decay=weight_decay,
                                      momentum=momentum, centered=centered, grad_scale=grad_scale), grad_dtype)

    def _state_names_for(self, gi):
        g = self.param_groups[gi]
        names = ["square_avg"]
        if g["momentum"] > 0:
            names.append("momentum_buffer")
        if g["centered"]:
            names.append("grad_avg")
        return tuple(names)

    def _step_gpu(self, gi, g, fg, start=0, end=None):
        end = fg.numel if end is None else end
        self._check(fg)
        sq = self._buf(gi, "square_avg")
        buf = self._buf(gi, "momentum_buffer") if g["momentum"] > 0 else None
        ga = self._buf(gi, "grad_avg") if g["centered"] else None
        lp, lpdt = self._lowp_args(fg, start)
        N.hip().rmsprop_step(self._at(fg.master, start), self._at(fg.grad, start), N.dtype_code(fg.grad.dtype),
                             self._at(sq, start), self._at(buf, start), self._at(ga, start), lp, lpdt, end - start,
                             float(g["lr"]), float(g["alpha"]), float(g["eps"]), float(g["weight_decay"]),
                             float(g["momentum"]), bool(g["centered"]), float(g["grad_scale"]),
                             N.stream_of(fg.master))

    def _step_cpu(self, gi, g, fg, start=0, end=None):
        sl = slice(start, fg.numel if end is None else end)
        p = fg.master[sl]
        d = fg.grad[sl].float() * g["grad_scale"]
        if g["weight_decay"] != 0:
            d = d + g["weight_decay"] * p
        sq = self._buf(gi, "square_avg")[sl]
        sq.mul_(g["alpha"]).addcmul_(d, d, value=1 - g["alpha"])
        if g["centered"]:
            ga = self._buf(gi, "grad_avg")[sl]
            ga.mul_(g["alpha"]).add_(d, alpha=1 - g["alpha"])
            avg = (sq - ga * ga).sqrt_().add_(g["eps"])
        else:
            avg = sq.sqrt().add_(g["eps"])
        if g["momentum"] > 0:
            buf = self._buf(gi, "momentum_buffer")[sl]
            buf.mul_(g["momentum"]).addcdiv_(d, avg)
            p.add_(buf, alpha=-g["lr"])
        else:
            p.addcdiv_(d, avg, value=-g["lr"])
        _sync_lowp(fg, sl)


def _sync_lowp(fg: FlatGroup, sl: slice) -> None:
    if fg.lowp is not None:
        fg.lowp[sl].copy_(fg.master[sl])


def make_optimizer(name: str, params, **kw) -> _FusedFlatOptimizer:
    """Factory used by the workload specs (``--optimizer SGD|Adam|AdamW|RMSprop``).
    ``grad_dtype`` (default fp32) is the precision of the flat gradient buffers."""
    key = name.lower()
    table = {"sgd": FusedSGD, "adam": FusedAdam, "adamw": FusedAdamW, "rmsprop": FusedRMSprop}
    if key not in table:
        raise ValueError(f"unknown optimizer {name!r}; expected one of {sorted(table)}")
    return table[key](params, **kw)
