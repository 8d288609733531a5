"""Fused multi-tensor SGD (torch.optim.SGD semantics, train.py:195-198) on the HIP path.

When every parameter of a group is a view of one flat arena and every ``.grad`` a view of one
flat gradient buffer at the same offsets (what ``FastSCNN`` produces), the whole step is ONE
kernel over the arena (one per contiguous run when frozen parameters or another group's tensors
sit inside the group's span: those are never touched).  Otherwise it falls back to one launch
per tensor (still the HIP kernel).
State keeps torch's ``momentum_buffer`` key so ``state_dict()`` interoperates.
"""
import torch

from . import _lib


def _flat_base(tensors):
    """(base tensor storage pointer, [offsets]) if all tensors are contiguous views of one
    storage, else None."""
    st = tensors[0].untyped_storage().data_ptr()
    offs = []
    for t in tensors:
        if not t.is_contiguous() or t.untyped_storage().data_ptr() != st:
            return None
        offs.append(t.storage_offset())
    return st, offs


def _runs(offs, numels, align=16):
    """Split tensors (sorted by offset) into maximal runs that tile a flat span with nothing but
    alignment padding between neighbours: [(lo, hi)] in elements.  A parameter of another group,
    or one without a gradient (frozen), that lies between two tensors breaks the run, so the
    fused launch never touches it (torch.optim.SGD skips grad-None parameters)."""
    order = sorted(range(len(offs)), key=lambda i: offs[i])
    runs = []
    lo = hi = None
    for i in order:
        o, n = offs[i], numels[i]
        if lo is not None and o == (hi + align - 1) // align * align:
            hi = o + n
            continue
        if lo is not None:
            runs.append((lo, hi))
        lo, hi = o, o + n
    if lo is not None:
        runs.append((lo, hi))
    return runs


class FusedSGD(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-2, momentum=0.0, dampening=0.0, weight_decay=0.0,
                 nesterov=False, grad_scale=1.0):
        if lr < 0.0:
            raise ValueError("Invalid learning rate: {}".format(lr))
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening,
                        weight_decay=weight_decay, nesterov=nesterov, grad_scale=grad_scale)
        super().__init__(params, defaults)
        self._aux = {}  # group index -> {"flat": momentum arena, "plan": cached fused plan}

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._aux = {}  # momentum buffers were replaced: rebuild the flat view on the next step

    def _launch(self, p, g, buf, n, group, first):
        _lib.call("fscnn_sgd", _lib.c_vp(p), _lib.c_vp(g), _lib.c_vp(buf), n,
                  _lib.c_float(group["lr"]), _lib.c_float(group["momentum"]),
                  _lib.c_float(group["dampening"]), _lib.c_float(group["weight_decay"]),
                  int(group["nesterov"]), int(first), _lib.c_float(group["grad_scale"]),
                  _lib.stream_ptr())

    def _launch_runs(self, pbase, gbase, flat, lo, runs, group, first):
        for a, b in runs:
            self._launch(pbase + a * 4, gbase + a * 4, flat.data_ptr() + (a - lo) * 4, b - a,
                         group, first)

    def _fast_step(self, gi, group):
        """Steady-state path: same parameter views as the cached fused plan and every grad a
        view of one base at the parameters' offsets (what FastSCNN's backward returns) -> one
        launch per contiguous run without re-deriving the plan.  False when it does not apply."""
        aux = self._aux.get(gi)
        plan = aux.get("plan") if aux else None
        params = group["params"]
        if plan is None or len(params) != plan["n"]:
            return False
        if params[0].data_ptr() != plan["p0"] or params[-1].data_ptr() != plan["p1"]:
            return False
        g0 = params[0].grad
        if g0 is None or g0.dtype != torch.float32:
            return False
        base = g0._base
        if base is None:
            return False
        offs = plan["offs"]
        for p, o in zip(params, offs):
            g = p.grad
            if g is None or g._base is not base or g.storage_offset() != o:
                return False
        gptr = base.untyped_storage().data_ptr()
        self._launch_runs(plan["pbase"], gptr, aux["flat"], plan["lo"], plan["runs"], group,
                          False)
        return True

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            if self._fast_step(gi, group):
                continue
            aux = self._aux.setdefault(gi, {})
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            for p in params:
                if not p.is_cuda or p.dtype != torch.float32:
                    raise RuntimeError("FusedSGD needs fp32 ROCm parameters")
            grads = [p.grad for p in params]
            first = any("momentum_buffer" not in self.state[p] for p in params)
            pb, gb = _flat_base([p.data for p in params]), _flat_base(grads)
            fused = (pb is not None and gb is not None and pb[1] == gb[1] and
                     all(p.grad.dtype == torch.float32 for p in params) and
                     not any(("momentum_buffer" in self.state[p]) != (not first) for p in params))
            if fused:
                runs = _runs(pb[1], [p.numel() for p in params])
                lo, hi = runs[0][0], runs[-1][1]
                flat = aux.get("flat")
                if flat is None or flat.numel() != hi - lo or first:
                    flat = torch.zeros(hi - lo, dtype=torch.float32, device=params[0].device)
                    aux["flat"] = flat
                    for o, p in zip(pb[1], params):
                        view = flat[o - lo:o - lo + p.numel()].view_as(p)
                        old = self.state[p].get("momentum_buffer")
                        if old is not None and not first:  # e.g. after load_state_dict
                            view.copy_(old)
                        self.state[p]["momentum_buffer"] = view
                # pointer base of element 0 of the storage: offsets are in elements
                self._launch_runs(pb[0], gb[0], flat, lo, runs, group, first)
                if len(params) == len(group["params"]):
                    aux["plan"] = {"n": len(params), "p0": params[0].data_ptr(),
                                   "p1": params[-1].data_ptr(), "offs": list(gb[1]),
                                   "pbase": pb[0], "lo": lo, "runs": runs}
                else:
                    aux.pop("plan", None)
            else:
                for p in params:
                    st = self.state[p]
                    f = "momentum_buffer" not in st
                    if f:
                        st["momentum_buffer"] = torch.zeros_like(p)
                    g = p.grad.float().contiguous()
                    self._launch(p.data_ptr(), g.data_ptr(), st["momentum_buffer"].data_ptr(),
                                 p.numel(), group, f)
        return loss
