"""The train.py step (train.py:77-97) for one process per GPU: forward on the fs2hip kernels
(fs2amd/training.py), FastSpeech2Loss, backward, gradient all-reduce, clip_grad_norm_,
ScheduledOptim.step_and_update_lr.

Data parallel: the reference uses nn.DataParallel in one process; here
each rank owns one GPU and its shard of the batch, and the only exchange is the mean all-reduce
of the 34.66 M fp32 gradients (138.6 MB) over RCCL. Two forms:

* eager steps (graph=False): DistributedDataParallel, bucketed and overlapped with the backward.
  Buckets are sized for xGMI rings: each bucket's all-reduce is a bandwidth-bound ring over 7
  point-to-point links, so a few large buckets (default 32 MB: five for the whole model) keep
  per-collective latency small against ~153 GB/s per link;
* graph=True: the whole step is captured as ONE HIP graph, RCCL collectives included. The
  gradients live in one flat fp32 buffer (every ``p.grad`` is a view of it, as DDP's
  gradient_as_bucket_view), zeroed at the start of each step; after the backward the buffer is
  all-reduced in ``bucket_mb`` slices (``world_size`` > 1 or ``ddp=True``) and scaled by
  1/world_size, then clip_grad_norm_ and the capturable fused Adam run inside the same graph.
  DDP's autograd hooks cannot be captured; this explicit form can.

PostNet BatchNorm running stats follow rank 0 (DataParallel's semantics: DDP broadcast_buffers,
or one coalesced broadcast per step in the graph form). Gradient clipping needs no extra
collective: after the all-reduce every rank holds the same gradients.
"""
import time

import torch
import torch.distributed as dist
import torch.nn as nn

from .data import loss_inputs
from .loss import FastSpeech2Loss
from .optimizer import ScheduledOptim
from .training import grad_sink


class TrainStep:
    """graph=True (fixed batch shapes): after ``warmup`` eager steps, run on the capture stream,
    the whole step — forward, loss, backward, gradient all-reduce, clip_grad_norm_, Adam — is
    captured once as a HIP graph and replayed; each call copies the batch into the graph's static
    input buffers, writes the step's Noam lr into the optimizer's lr tensor and replays (one launch
    instead of ~1,600). A batch with other shapes runs the same step body eagerly (same flat
    gradient buffer, zeroed first: nothing a replay left behind is accumulated into it).

    ``optimizer``: an existing ScheduledOptim (e.g. the one ``get_model(train=True)`` restored from
    a checkpoint, utils/model.py:15-28) whose Adam state and step count this step continues.
    Returned losses are fresh tensors on every call (the graph's static outputs are copied)."""

    def __init__(self, model, preprocess_config, model_config, train_config, device=None, world_size=1,
                 bucket_mb=32, current_step=0, graph=False, warmup=3, ddp=None, optimizer=None, flat_grads=None):
        self.model = model.train()
        self.net = model
        self.device = device
        self.world_size = world_size
        self.bucket_mb = bucket_mb
        self.graph_mode = bool(graph) and device is not None and device.type == "cuda"
        self.warmup = warmup
        self._graph = None
        if ddp is None:
            ddp = world_size > 1
        self.reduce = bool(ddp) or world_size > 1  # gradient all-reduce in the step
        # flat gradient buffer + explicit all-reduce: always with graph=True; flat_grads=True runs the
        # same step body eagerly (the N-rank test of the graph form's reduction on CPU / gloo)
        self.flat = self.graph_mode if flat_grads is None else (bool(flat_grads) or self.graph_mode)
        if ddp and not self.flat:  # ddp=True at world size 1 still runs DDP's bucketed all-reduce
            ids = [device.index] if device is not None and device.type == "cuda" else None
            self.net = nn.parallel.DistributedDataParallel(model, device_ids=ids, bucket_cap_mb=bucket_mb,
                                                           gradient_as_bucket_view=True, broadcast_buffers=True)
        self.loss = FastSpeech2Loss(preprocess_config, model_config)
        if optimizer is not None:
            current_step = optimizer.current_step
        self.optimizer = ScheduledOptim(model, train_config, model_config, current_step, capturable=self.graph_mode)
        if optimizer is not None:
            self.optimizer.load_state_dict(optimizer._optimizer.state_dict())
        opt = train_config["optimizer"]
        self.grad_acc_step = opt["grad_acc_step"]
        self.grad_clip_thresh = opt["grad_clip_thresh"]
        self.step_no = current_step + 1
        self._flat = None
        self._stream = None
        self._closed = False
        self._acc_pending = 0
        self._calls = 0  # steps this TrainStep ran (warm-up counts these, not the resumed step number)
        self._fused_adam = False
        if self.flat:
            self._setup_flat_grads()
            # every optimizer parameter has its gradient in the flat buffer
            # (frozen parameters, e.g. the position-encoding tables, never get a gradient: torch's Adam
            # skips them, and so does the flat update)
            inflat = {id(p) for p in self._flat_params}
            self._fused_adam = (self.optimizer.flat_step_ok() and
                                all(id(p) in inflat or not p.requires_grad
                                    for p in self.optimizer._optimizer.param_groups[0]["params"]))
        if self.graph_mode:
            self._stream = torch.cuda.Stream(device)

    def __call__(self, batch):
        """One step on this rank's shard (a dict of forward kwargs + mels / targets on the device).
        Returns the 6 loss tensors (train.py:85-86)."""
        if self._closed:
            raise RuntimeError("TrainStep: step after close()")
        if self.graph_mode and self.grad_acc_step == 1:
            return self._graphed(batch)
        if self.flat:
            if self.grad_acc_step > 1:
                return self._flat_accumulate(batch)
            self.optimizer._update_learning_rate()
            losses = [l.detach() for l in self._step_body(batch)]
            self.step_no += 1
            return losses
        return self._eager(batch)

    def close(self):
        """Release the captured step graph (it holds RCCL all-reduces on the process group's
        communicator), its static inputs / outputs and the DDP reducer, after the device has
        drained. Call before ``dist.destroy_process_group()``: tearing the communicator down
        while a graph that captured collectives on it is alive aborts the process (round-3
        GPU suite). Idempotent; the model keeps its parameters (gradients are detached from the
        flat buffer)."""
        if self._closed:
            return
        if self.device is not None and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        if self._graph is not None:
            g = self._graph[1]
            self._graph = None
            g.reset()
        if self._flat is not None:
            for p in self.model.parameters():
                p.grad = None
            self._flat = None
            self._buckets = []
        self.net = self.model
        self._stream = None
        self._closed = True
        if self.device is not None and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

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

    # ---- flat gradients + explicit all-reduce (graph form) -------------------------------------
    def _setup_flat_grads(self):
        params = [p for p in self.model.parameters() if p.requires_grad]
        self._flat_params = params
        # each gradient starts on a 16-byte boundary (the fused Adam's vector loads); the few gap
        # elements stay zero (all-reduced and counted in the norm as zeros)
        offs, n = [], 0
        for p in params:
            offs.append(n)
            n += (p.numel() + 3) // 4 * 4
        self._flat = torch.zeros(n, dtype=torch.float32, device=params[0].device)
        for p, off in zip(params, offs):
            p.grad = self._flat[off:off + p.numel()].view_as(p)
        step = max(1, int(self.bucket_mb * (1 << 20) // 4))
        self._buckets = [self._flat[i:i + step] for i in range(0, n, step)]
        self._bn_buffers = [b for name, b in self.model.named_buffers()
                            if b.is_floating_point() and ("running_" in name)]

    def _reduce_grads(self):
        if not self.reduce:
            return
        for b in self._buckets:
            dist.all_reduce(b)
        if self.world_size > 1:
            self._flat.mul_(1.0 / self.world_size)

    def _sync_buffers(self):
        if self.world_size > 1 and self._bn_buffers:
            flat = torch.cat([b.reshape(-1) for b in self._bn_buffers])
            dist.broadcast(flat, 0)
            torch._foreach_copy_(self._bn_buffers, list(flat.split([b.numel() for b in self._bn_buffers])))

    def _flat_accumulate(self, batch):
        """grad_acc_step > 1 on the flat buffer (train.py:89-97): the loss is divided by
        grad_acc_step and its gradient accumulated; every grad_acc_step-th call reduces, clips,
        takes the Noam lr step and zeroes the buffer (eager launches: a replayed graph would
        re-zero the buffer each call)."""
        if self._acc_pending == 0:
            self._flat.zero_()
            self._sync_buffers()
        output = self.net(**batch)
        losses = self.loss(loss_inputs(batch), output)
        with grad_sink():
            (losses[0] / self.grad_acc_step).backward()
        self._acc_pending += 1
        if self.step_no % self.grad_acc_step == 0:
            self._reduce_grads()
            self.optimizer._update_learning_rate()
            self._clip_and_step()
            self._acc_pending = 0
        self.step_no += 1
        return [l.detach() for l in losses]

    def _step_body(self, batch):
        """zero grads, forward, loss, backward, all-reduce, clip, Adam: the captured step."""
        self._flat.zero_()
        self._sync_buffers()
        output = self.net(**batch)
        losses = self.loss(loss_inputs(batch), output)
        with grad_sink():  # the fused blocks accumulate straight into the flat buffer's views
            losses[0].backward()
        self._reduce_grads()
        self._clip_and_step()
        return losses

    def _clip_and_step(self):
        """clip_grad_norm_ + Adam: on the flat buffer in two launches (fs2_adam_flat) when the
        optimizer allows it, else torch's."""
        if self._fused_adam:
            self.optimizer.flat_step(self._flat, self._flat_params, self.grad_clip_thresh)
        else:
            nn.utils.clip_grad_norm_(self.model.parameters(), self.grad_clip_thresh)
            self.optimizer._optimizer.step()

    # ---- whole-step HIP graph --------------------------------------------------------------------
    @staticmethod
    def _sig(batch):
        return tuple((k, tuple(v.shape), v.dtype) if torch.is_tensor(v) else (k, v) for k, v in sorted(batch.items()))

    def _on_stream(self, fn):
        """Run fn on the capture stream (warm-up and eager fallbacks: the autograd engine then
        runs every backward on the stream the graph is captured on)."""
        cur = torch.cuda.current_stream(self.device)
        self._stream.wait_stream(cur)
        with torch.cuda.stream(self._stream):
            out = fn()
        cur.wait_stream(self._stream)
        return out

    @staticmethod
    def _static_inputs(batch):
        """The captured step's static inputs as views of ONE byte slab (widest element type first, so
        every view is aligned): a later batch is copied in by one concatenating launch instead of one
        copy per tensor (~5 us each inside the step). Returns (static dict, (key order, slab))."""
        order = sorted((k for k, v in batch.items() if torch.is_tensor(v)), key=lambda k: -batch[k].element_size())
        flat = [batch[k].contiguous().view(-1).view(torch.uint8) for k in order]
        slab = torch.cat(flat)
        static = dict(batch)
        off = 0
        for k, f in zip(order, flat):
            n = f.numel()
            static[k] = slab[off:off + n].view(batch[k].dtype).view(batch[k].shape)
            off += n
        return static, (order, slab)

    def _graphed(self, batch):
        # warm-up by the calls of THIS TrainStep (at least one eager step, whatever `warmup` says): a
        # step resumed from a checkpoint (current_step > warmup) still runs the lazy one-time setup
        # (fused-Adam plan, dropout seed: synchronous host copies, illegal inside a capture) eagerly
        self._calls += 1
        if self._calls <= max(1, self.warmup) or (self._graph is not None and self._sig(batch) != self._graph[0]):
            # eager step body (same flat buffer, zeroed inside): detached losses, so no autograd
            # graph of a warm-up step outlives it into the capture
            self.optimizer._update_learning_rate()
            losses = self._on_stream(lambda: [l.detach() for l in self._step_body(batch)])
            self.step_no += 1
            return losses
        if self._graph is None:
            if dist.is_available() and dist.is_initialized():
                # let the process group's watchdog retire the warm-up steps' collectives first: HIP
                # rejects an event query once the event's stream (RCCL's, joined by the captured
                # all-reduces) is capturing, and the watchdog aborts the process on that error
                torch.cuda.synchronize(self.device)
                time.sleep(0.5)
            static, self._slab = self._static_inputs(batch)
            self.optimizer._update_learning_rate()
            g = torch.cuda.CUDAGraph()
            cur = torch.cuda.current_stream(self.device)
            self._stream.wait_stream(cur)
            # thread_local: with an RCCL process group, its watchdog thread queries events while
            # this thread captures; under the default "global" mode such a call from ANY thread
            # invalidates the capture and capture_end aborts (intermittently: it depends on the
            # watchdog's timing). The warm-up steps ran on this stream with detached losses, so no
            # autograd node of theirs (AccumulateGrad bound to another stream) reaches the capture.
            with torch.cuda.graph(g, stream=self._stream, capture_error_mode="thread_local"):
                losses = [l.detach() for l in self._step_body(static)]
            cur.wait_stream(self._stream)
            self._graph = (self._sig(batch), g, static, losses)
            g.replay()  # the captured step has not run yet: this is its execution
            self.step_no += 1
            return list(torch.stack(losses).unbind())
        _, g, static, losses = self._graph
        order, slab = self._slab
        if all(batch[k].device == slab.device for k in order):
            # one launch: the batch's bytes into the slab the static inputs are views of
            torch.cat([batch[k].contiguous().view(-1).view(torch.uint8) for k in order], out=slab)
        else:
            for k in order:
                static[k].copy_(batch[k], non_blocking=True)
        self.optimizer._update_learning_rate()
        g.replay()
        self.step_no += 1
        return list(torch.stack(losses).unbind())
