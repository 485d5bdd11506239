"""torch.optim.AdamW (the reference's optimizer, src/main.py:416-457) whose CUDA step runs csrc/optim.hip.

Same parameter groups, hyper-parameters, state layout (state[p] = {"step": fp32 device scalar, "exp_avg",
"exp_avg_sq"}) and state_dict as torch's fused AdamW, and the same GradScaler contract (`grad_scale` / `found_inf`
set on the optimizer by GradScaler.step, steps rolled back when found_inf). torch's fused kernel deals ~64 K
elements to a block, so the head's ~3 M parameters ran on ~50 blocks for ~0.45 ms per step; rdx_adamw_many gives
every 4096 elements a block. Anything the kernel does not cover (CPU tensors, amsgrad, maximize, non-fp32 or
non-contiguous tensors) takes torch's own AdamW step.
"""
import ctypes

import torch

from ._lib import check, lib, ptr_array


class AdamW(torch.optim.AdamW):
    _step_supports_amp_scaling = True

    def __init__(self, params, **kw):
        kw.pop("fused", None)
        kw.pop("foreach", None)
        # the group flags torch's fused AdamW saves: a checkpoint of this optimizer resumed under torch's own
        # (RADHIP_ADAMW=0) keeps the fused form, the one that takes GradScaler's grad_scale / found_inf
        super().__init__(params, fused=True, **kw)

    def load_state_dict(self, state_dict):
        """torch's load, then this optimizer's own form: the groups keep torch's fused flags (a state_dict of torch's
        non-fused AdamW brings fused=False), every step count a device fp32 scalar, and every state tensor a copy of
        its own (torch's load keeps a tensor already of the right device and dtype as the very object of the source
        state_dict, so an optimizer loaded from another live one would share its moments and step counts)."""
        super().load_state_dict(state_dict)
        self._tables = {}
        for group in self.param_groups:
            group["fused"] = True
            group["foreach"] = None
            for p in group["params"]:
                st = self.state.get(p)
                if not st:
                    continue
                for k, v in list(st.items()):
                    if torch.is_tensor(v):
                        st[k] = v.detach().clone()
                if torch.is_tensor(st.get("step")) and p.is_cuda:
                    st["step"] = st["step"].to(device=p.device, dtype=torch.float32)

    def _covered(self, group, ps):
        return (all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.grad.dtype == torch.float32
                    and p.grad.is_contiguous() and not p.grad.is_sparse for p in ps)
                and not group["amsgrad"] and not group["maximize"] and not group.get("differentiable", False)
                and not torch.is_tensor(group["lr"]))

    def _launch_table(self, gi, group, ps):
        """Per group: the step counters as views of one flat fp32 device tensor (the increment and GradScaler's
        rollback are one launch each, where torch's per-tensor _foreach_add_ / _foreach_sub_ over a few hundred
        scalars cost ~0.6 ms of host time apiece) and the kernel's pointer arrays, rebuilt only when the group's
        parameters, gradients or state tensors change (a loaded state_dict, a .grad re-bound)."""
        # the table keeps every keyed object alive (ids cannot be reused while it holds them)
        key = tuple((id(p), id(p.grad), p.data_ptr(), p.grad.data_ptr()) for p in ps)
        tab = self._tables.get(gi)
        if tab is not None and tab["key"] == key and all(
                self.state[p].get("step") is s for p, s in zip(ps, tab["ss"])):
            return tab
        ms, vs, ss = [], [], []
        for p in ps:
            st = self.state[p]
            if len(st) == 0:
                st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            ms.append(st["exp_avg"])
            vs.append(st["exp_avg_sq"])
            # a loaded state_dict may hold the step as a CPU scalar (torch's non-fused AdamW, or
            # map_location="cpu"); the kernel reads it on the device, as torch's fused step does
            ss.append(st["step"].to(device=p.device, dtype=torch.float32).reshape(()))
        flat = torch.stack(ss)
        for i, p in enumerate(ps):
            self.state[p]["step"] = flat[i]
        ss = [self.state[p]["step"] for p in ps]
        mx = int(lib().rdx_adamw_many_max())
        chunks = []
        for i in range(0, len(ps), mx):
            sl = slice(i, i + mx)
            n = len(ps[sl])
            chunks.append((n, ptr_array([p.data_ptr() for p in ps[sl]]), ptr_array([p.grad.data_ptr() for p in ps[sl]]),
                           ptr_array([t.data_ptr() for t in ms[sl]]), ptr_array([t.data_ptr() for t in vs[sl]]),
                           ptr_array([t.data_ptr() for t in ss[sl]]), (ctypes.c_int64 * n)(*[p.numel() for p in ps[sl]])))
        tab = {"key": key, "ss": ss, "flat": flat, "chunks": chunks, "keep": (ps, [p.grad for p in ps], ms, vs)}
        self._tables[gi] = tab
        return tab

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        grad_scale = getattr(self, "grad_scale", None)
        found_inf = getattr(self, "found_inf", None)
        if not hasattr(self, "_tables"):
            self._tables = {}
        for gi, group in enumerate(self.param_groups):
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            if not self._covered(group, ps):
                self._torch_step(group, ps, grad_scale, found_inf)
                continue
            tab = self._launch_table(gi, group, ps)
            tab["flat"].add_(1)
            b1, b2 = group["betas"]
            stream = torch.cuda.current_stream(ps[0].device).cuda_stream
            gsp = grad_scale.data_ptr() if grad_scale is not None else None
            fip = found_inf.data_ptr() if found_inf is not None else None
            for n, pp, gp, mp, vp, sp, numel in tab["chunks"]:
                check(lib().rdx_adamw_many(n, pp, gp, mp, vp, sp, numel, float(group["lr"]), float(b1), float(b2),
                                           float(group["weight_decay"]), float(group["eps"]), gsp, fip, stream),
                      "adamw_many")
            if found_inf is not None:
                tab["flat"].sub_(found_inf)
        return loss

    def _torch_step(self, group, ps, grad_scale, found_inf):
        """torch's own AdamW update for a group the kernel does not cover (same state layout)."""
        from torch.optim.adamw import adamw
        ms, vs, mxs, ss = [], [], [], []
        for p in ps:
            st = self.state[p]
            if len(st) == 0:
                st["step"] = torch.zeros((), dtype=torch.float32, device=p.device) if p.is_cuda else torch.tensor(0.0)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                if group["amsgrad"]:
                    st["max_exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            ms.append(st["exp_avg"])
            vs.append(st["exp_avg_sq"])
            ss.append(st["step"])
            if group["amsgrad"]:
                mxs.append(st["max_exp_avg_sq"])
        b1, b2 = group["betas"]
        fused = all(p.is_cuda for p in ps)      # torch's fused form is the one that takes grad_scale / found_inf
        adamw(ps, [p.grad for p in ps], ms, vs, mxs, ss, foreach=False, capturable=False, differentiable=False,
              fused=fused or None, grad_scale=grad_scale, found_inf=found_inf, amsgrad=group["amsgrad"], beta1=b1, beta2=b2,
              lr=group["lr"], weight_decay=group["weight_decay"], eps=group["eps"], maximize=group["maximize"],
              has_complex=False)
