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
