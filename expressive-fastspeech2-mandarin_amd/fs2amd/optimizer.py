"""ScheduledOptim: Adam with the Noam warm-up / inverse-sqrt schedule and step annealing
(model/optimizer.py:5-51): lr = d_model^-0.5 * min(step^-0.5, warmup^-1.5 * step)
* anneal_rate^(#anneal_steps passed)."""
import numpy as np
import torch


class ScheduledOptim:
    def __init__(self, model, train_config, model_config, current_step, capturable=False):
        """capturable=True (GPU only): Adam keeps its step count and the learning rate in device
        tensors, so a HIP graph that captured optimizer.step() replays with each step's Noam lr
        (written into the lr tensor before the replay) — fs2amd.trainer.TrainStep(graph=True)."""
        opt = train_config["optimizer"]
        params = [p for p in model.parameters()]
        fused = bool(params) and all(p.is_cuda for p in params)  # one multi-tensor kernel per step on the GPU
        extra = {}
        if capturable and fused:
            extra = dict(capturable=True, lr=torch.tensor(1e-3, device=params[0].device))
        self._optimizer = torch.optim.Adam(params, betas=opt["betas"], eps=opt["eps"],
                                           weight_decay=opt["weight_decay"], fused=fused, **extra)
        self.n_warmup_steps = opt["warm_up_step"]
        self.anneal_steps = opt["anneal_steps"]
        self.anneal_rate = opt["anneal_rate"]
        self.current_step = current_step
        self.init_lr = np.power(model_config["transformer"]["encoder_hidden"], -0.5)

    # ---- clip + Adam over a flat gradient buffer in two launches (fs2_adam_flat) -----------------
    def flat_step_ok(self):
        """The fused flat update applies: one param group, plain Adam (no amsgrad / maximize /
        differentiable), every parameter on the GPU; FS2_FUSED_ADAM=0 disables it."""
        import os
        if os.environ.get("FS2_FUSED_ADAM", "1") == "0":
            return False
        gs = self._optimizer.param_groups
        if len(gs) != 1:
            return False
        g = gs[0]
        return (not g.get("amsgrad", False) and not g.get("maximize", False) and not g.get("differentiable", False)
                and all(p.is_cuda and p.dtype == torch.float32 for p in g["params"]))

    def flat_step(self, flat, params, max_norm):
        """clip_grad_norm_(params, max_norm) + Adam.step() where params' gradients are views of
        ``flat`` in increasing order, each starting on a 16-byte boundary (fs2amd.trainer's buffer;
        gap elements between them stay zero). The optimizer state is torch's own (exp_avg,
        exp_avg_sq, a float32 device step per parameter; created here if absent, outside capture),
        so state_dict / checkpoints are unchanged."""
        import ctypes
        from . import _lib as L
        from . import ops
        opt = self._optimizer
        group = opt.param_groups[0]
        key = (flat.data_ptr(),) + tuple(p.data_ptr() for p in params)
        plan = getattr(self, "_flat_plan", None)
        states = []
        for p in params:
            st = opt.state[p]
            if len(st) == 0:
                st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            states.append(st)
        key += tuple(st["exp_avg"].data_ptr() + st["exp_avg_sq"].data_ptr() + st["step"].data_ptr() for st in states)
        if plan is None or plan[0] != key:
            arr = (L.AdamParam * len(params))()
            base, end = flat.data_ptr(), 0
            for d, p, st in zip(arr, params, states):
                if not (p.is_contiguous() and st["exp_avg"].is_contiguous() and st["exp_avg_sq"].is_contiguous()):
                    raise RuntimeError("fs2amd: fused Adam needs contiguous parameters and state")
                if st["step"].device != p.device or st["step"].dtype != torch.float32:
                    st["step"] = st["step"].to(device=p.device, dtype=torch.float32)
                d.p, d.m, d.v, d.step = (p.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                                         st["step"].data_ptr())
                g = p.grad
                if g is None or not g.is_contiguous() or not (base <= g.data_ptr() < base + 4 * flat.numel()):
                    raise RuntimeError("fs2amd: every parameter's gradient must be a view of the flat buffer")
                d.off, d.numel = (g.data_ptr() - base) // 4, p.numel()
                ptrs = (g.data_ptr(), d.p, d.m, d.v)
                if any(x % 16 for x in ptrs) or d.off < end:
                    raise RuntimeError("fs2amd: fused Adam needs 16-byte aligned, increasing, disjoint gradient views")
                end = d.off + d.numel
            dev = torch.frombuffer(bytearray(bytes(memoryview(arr).cast("B"))), dtype=torch.uint8).to(flat.device)
            ws = torch.empty(L.load().fs2_adam_ws_bytes() // 4, device=flat.device, dtype=torch.float32)
            plan = self._flat_plan = (key, dev, ws, len(params))
        _, dev, ws, n = plan
        lr = group["lr"]
        lr_dev = ctypes.c_void_p(lr.data_ptr()) if torch.is_tensor(lr) else None
        b1, b2 = group["betas"]
        L.check(L.load().fs2_adam_flat(ctypes.c_void_p(flat.data_ptr()), flat.numel(), ctypes.c_void_p(dev.data_ptr()),
                                       n, lr_dev, float(lr) if not torch.is_tensor(lr) else 0.0, float(b1), float(b2),
                                       float(group["eps"]), float(group["weight_decay"]),
                                       float(max_norm) if max_norm is not None else 0.0,
                                       ctypes.c_void_p(ws.data_ptr()), ws.numel() * 4, ops._stream(flat)),
                "fs2_adam_flat")

    def step_and_update_lr(self):
        self._update_learning_rate()
        self._optimizer.step()

    def zero_grad(self):
        self._optimizer.zero_grad()

    def load_state_dict(self, state):
        self._optimizer.load_state_dict(state)

    def _get_lr_scale(self):
        lr = np.min([np.power(self.current_step, -0.5), np.power(self.n_warmup_steps, -1.5) * self.current_step])
        for s in self.anneal_steps:
            if self.current_step > s:
                lr = lr * self.anneal_rate
        return lr

    def _update_learning_rate(self):
        self.current_step += 1
        lr = self.init_lr * self._get_lr_scale()
        for group in self._optimizer.param_groups:
            if torch.is_tensor(group["lr"]):
                group["lr"].fill_(float(lr))  # capturable: the graph reads the lr from this tensor
            else:
                group["lr"] = lr
