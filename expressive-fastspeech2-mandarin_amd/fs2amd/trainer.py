"""The train.py step (train.py:77-97) for one process per GPU: forward on the fs2hip kernels
(fs2amd/training.py), FastSpeech2Loss, backward, gradient all-reduce, clip_grad_norm_,
ScheduledOptim.step_and_update_lr.

Data parallel: the reference uses nn.DataParallel in one process; here
each rank owns one GPU and its shard of the batch, and the only exchange is the mean all-reduce
of the 34.66 M fp32 gradients (138.6 MB) over RCCL, bucketed and overlapped with the backward by
DistributedDataParallel. Buckets are sized for xGMI rings: each bucket's all-reduce is a
bandwidth-bound ring over 7 point-to-point links, so a few large buckets (default 32 MB: five
for the whole model) keep per-collective latency small against ~153 GB/s per link, while still
letting the last decoder layers' gradients start reducing while the encoder's backward runs.
PostNet BatchNorm running stats are broadcast from rank 0 every forward (broadcast_buffers),
DataParallel's semantics. Gradient clipping needs no extra collective: after the all-reduce every
rank holds the same gradients.
"""
import torch
import torch.nn as nn

from .data import loss_inputs
from .loss import FastSpeech2Loss
from .optimizer import ScheduledOptim


class TrainStep:
    """graph=True (one process, fixed batch shapes): after ``warmup`` eager steps the whole step —
    forward, loss, backward, clip_grad_norm_, Adam — is captured once as a HIP graph and replayed;
    each call copies the batch into the graph's static input buffers, writes the step's Noam lr
    into the optimizer's lr tensor and replays (one launch instead of ~1,600). A batch with other
    shapes falls back to an eager step."""

    def __init__(self, model, preprocess_config, model_config, train_config, device=None, world_size=1,
                 bucket_mb=32, current_step=0, graph=False, warmup=3, ddp=None):
        self.model = model.train()
        self.net = model
        self.graph_mode = bool(graph) and world_size == 1 and device is not None and device.type == "cuda"
        self.warmup = warmup
        self._graph = None
        if ddp is None:
            ddp = world_size > 1
        if ddp:  # ddp=True at world size 1 still runs DDP's bucketed all-reduce (the RCCL path on one GPU)
            self.graph_mode = False
            ids = [device.index] if device is not None and device.type == "cuda" else None
            self.net = nn.parallel.DistributedDataParallel(model, device_ids=ids, bucket_cap_mb=bucket_mb,
                                                           gradient_as_bucket_view=True, broadcast_buffers=True)
        self.loss = FastSpeech2Loss(preprocess_config, model_config)
        self.optimizer = ScheduledOptim(model, train_config, model_config, current_step, capturable=self.graph_mode)
        opt = train_config["optimizer"]
        self.grad_acc_step = opt["grad_acc_step"]
        self.grad_clip_thresh = opt["grad_clip_thresh"]
        self.step_no = current_step + 1

    def __call__(self, batch):
        """One step on this rank's shard (a dict of forward kwargs + mels / targets on the device).
        Returns the 6 loss tensors (train.py:85-86)."""
        if self.graph_mode and self.grad_acc_step == 1:
            return self._graphed(batch)
        return self._eager(batch)

    def _eager(self, batch):
        output = self.net(**batch)
        losses = self.loss(loss_inputs(batch), output)
        (losses[0] / self.grad_acc_step).backward()
        if self.step_no % self.grad_acc_step == 0:
            nn.utils.clip_grad_norm_(self.model.parameters(), self.grad_clip_thresh)
            self.optimizer.step_and_update_lr()
            self.optimizer.zero_grad()
        self.step_no += 1
        return losses

    # ---- whole-step HIP graph --------------------------------------------------------------------
    @staticmethod
    def _sig(batch):
        return tuple((k, tuple(v.shape), v.dtype) if torch.is_tensor(v) else (k, v) for k, v in sorted(batch.items()))

    def _step_body(self, batch):
        output = self.net(**batch)
        losses = self.loss(loss_inputs(batch), output)
        losses[0].backward()
        nn.utils.clip_grad_norm_(self.model.parameters(), self.grad_clip_thresh)
        self.optimizer._optimizer.step()
        return losses

    def _graphed(self, batch):
        if self.step_no <= self.warmup or (self._graph is not None and self._sig(batch) != self._graph[0]):
            return self._eager(batch)
        if self._graph is None:
            static = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in batch.items()}
            self.optimizer.zero_grad()
            self.optimizer._update_learning_rate()
            dev = next(self.model.parameters()).device
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):  # zero_grad(set_to_none) above: the backward WRITES every grad
                losses = self._step_body(static)
            self._graph = (self._sig(batch), g, static, losses)
            g.replay()  # the captured step has not run yet: this is its execution
            self.step_no += 1
            return losses
        _, g, static, losses = self._graph
        for k, v in batch.items():
            if torch.is_tensor(v):
                static[k].copy_(v, non_blocking=True)
        self.optimizer._update_learning_rate()
        g.replay()
        self.step_no += 1
        return losses
