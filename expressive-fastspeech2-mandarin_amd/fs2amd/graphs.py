"""Free-running synthesis as two captured HIP graphs around its one host read.

The synthesis call of synthesize_chinese_pinyin.py:140-145 is an eval forward with predicted
durations: the decoder length T_out = max(mel_len) is known only after the duration predictor
has run, so the path has one device->host read (runtime.host_meta) and cannot be ONE graph.
:class:`SynthGraphs` captures the two halves:

* stage 1 (keyed by B, L_max and the control values; an LRU of ``max_stage1`` graphs): token
  embedding + PE, the encoder, the
  variance adaptor and the LengthRegulator scan (duration rounding, cumulative frames, mel_len),
  plus the int32 meta vector [max(mel_len), sum(mel_len), out-of-vocabulary count];
* the host reads the meta vector (one sync), raises IndexError on bad ids;
* stage 2 (keyed by stage 1's key, the T bucket and the decoder's row bucket; an LRU of
  ``max_stage2`` graphs): the LengthRegulator gather + PE and the decoder on packed rows
  (runtime.decode_packed), captured for T_b = T_out rounded up to a multiple of ``t_step``: the
  packed rows and their layout do not depend on T beyond T >= max(mel_len) (the padded-row map
  and the grids' early-exiting tails do), so one graph serves every batch of the bucket and a
  stream of distinct batches stops recapturing;
* the T_out-shaped tail, issued eagerly behind the stage-2 replay (the host enqueues it while
  the GPU runs the decoder): the packed layout over T_out, mel_linear into [B, T_out, n_mel], the
  PostNet (valid-region form when the batch is mostly padding, runtime._postnet) and the mel mask.
* speculative stage 2 (round 6): the decoder graph of the buckets recent calls of the same stage-1
  key needed is replayed right behind stage 1, BEFORE the host has read the meta vector, so the GPU
  does not idle through the read (~50 us per call). After the read the speculation is kept when the
  call fits it -- T_out within its T bucket, the active rows within its row bucket, and the same
  decoder launch forms (runtime.decoder_forms: the FFN tile / split choice is the only thing the
  row bucket changes in the arithmetic), so the outputs are bit-identical to the exact bucket's --,
  else the exact graph replays after it (the speculative one only wrote its own buffers).
  FS2_SYNTH_SPEC=0 turns it off.
  Where the packed path does not apply (frame-level variance, a kernel-3 w_2) stage 2 is the whole
  of runtime._stage2, keyed by the exact T_out.

Each entry keeps the weight pack it was captured against (model.packed): when the weights change the
pack is rebuilt, and the stale graphs are dropped and recaptured on the next call. Each call
copies the batch into stage 1's static inputs and replays; the returned 10-tuple is
the reference's (fastspeech2.py:138-148), freshly allocated: stage 1's outputs leave the graph's
buffers through ONE concatenating copy into a fresh slab (views of it are returned), the tail
allocates its own.
Graph replay replaces ~100 kernel launches and the host bubbles around the read; numerics are
those of the eager path (same kernels, same order).
"""
import os
from collections import OrderedDict, deque
from types import SimpleNamespace

import torch

from . import ops
from . import runtime as R


def _fresh(srcs):
    """Fresh copies of the graph-owned tensors ``srcs`` in ONE launch (a byte-level torch.cat into a
    new slab; the returned tensors are views of it), widest element type first so every view is
    aligned. Replaces one copy launch per tensor."""
    order = sorted(range(len(srcs)), key=lambda i: -srcs[i].element_size())
    flat = [srcs[i].contiguous().view(-1).view(torch.uint8) for i in order]
    slab = torch.cat(flat)
    outs = [None] * len(srcs)
    off = 0
    for i, f in zip(order, flat):
        n = f.numel()
        outs[i] = slab[off:off + n].view(srcs[i].dtype).view(srcs[i].shape)
        off += n
    return outs


def _spin_until_landed(meta_np, budget_s=0.05):
    """Poll the pinned meta vector (a numpy view of it: an element read is ~0.1 us where a tensor
    index + int() is several) until its first entry leaves -1 (the device->host copy landed), for
    at most budget_s (the caller's stream synchronize covers the rest)."""
    import time

    t_end = time.perf_counter() + budget_s
    while meta_np[0] == -1 and time.perf_counter() < t_end:
        pass


class SynthGraphs:
    def __init__(self, model, max_stage2=16, max_stage1=4, t_step=64, speculate=None, history=8):
        self.model = model
        self.max_stage2 = max_stage2
        self.max_stage1 = max_stage1
        self.t_step = t_step
        self.speculate = os.environ.get("FS2_SYNTH_SPEC", "1") != "0" if speculate is None else speculate
        self._g1 = OrderedDict()
        self._g2 = OrderedDict()
        self._hist = {}  # key1 -> the exact (T bucket, row bucket, decoder forms) of recent calls
        self._history = history
        self.captures = 0
        self.spec_hits = 0
        self.spec_misses = 0

    def _spec_key(self, key1):
        """The speculative stage-2 buckets for key1: the largest T and row buckets among the recent
        calls that had the latest call's decoder forms (a call with other forms cannot reuse them)."""
        h = self._hist.get(key1)
        if not h:
            return None
        forms = h[-1][2]
        same = [x for x in h if x[2] == forms]
        return max(x[0] for x in same), max(x[1] for x in same), forms

    def _drop_stage1(self, key1):
        """Drop a stage-1 graph and every stage-2 graph captured on its outputs (key2 starts with
        key1): those read the dropped graph's buffers."""
        self._g1.pop(key1, None)
        self._hist.pop(key1, None)
        for k in [k for k in self._g2 if k[:len(key1)] == key1]:
            del self._g2[k]

    def close(self):
        """Release every captured graph (and the memory pools they hold)."""
        torch.cuda.synchronize()
        self._g1.clear()
        self._g2.clear()

    @staticmethod
    def _inputs(dev, speakers, emotions, arousals, valences, texts, src_lens, p_targets, e_targets):
        i64 = lambda t: None if t is None else torch.as_tensor(t).to(device=dev, dtype=torch.int64).contiguous()
        f32 = lambda t: None if t is None else t.to(device=dev, dtype=torch.float32).contiguous()
        return dict(speakers=i64(speakers), emotions=i64(emotions), arousals=i64(arousals), valences=i64(valences),
                    texts=i64(texts), src_lens=i64(src_lens), p_targets=f32(p_targets), e_targets=f32(e_targets))

    def _stage1_body(self, P, va, s, Lx, controls):
        p_c, e_c, d_c = controls
        g = SimpleNamespace(speakers=s["speakers"], emotions=s["emotions"], arousals=s["arousals"],
                            valences=s["valences"], texts=s["texts"], lens_src=s["src_lens"], Lx=Lx,
                            p_targets=s["p_targets"], e_targets=s["e_targets"], d_targets=None, mel_lens=None,
                            mask_out=None)
        src_masks = None
        if R.embed_block_ok(P, Lx):
            # the first encoder block's launch builds its input and writes the source mask
            src_masks = torch.empty(s["texts"].shape[0], Lx, device=s["texts"].device, dtype=torch.bool)
            g.mask_out = (src_masks, None, None)
        st = R._stage1(P, va, g, p_c, d_c)
        if R.packed_stage2_ok(P, st, st.x) and R.lr_proj_ok(P, st.x):
            # the decoder's first Q|K|V on the phoneme rows does not depend on T: it runs here,
            # under the host read, instead of opening stage 2
            st.xw = R.phoneme_qkv0(P, st.x)
        if src_masks is None:
            src_masks = R._mask(s["src_lens"], Lx)
        return g, st, src_masks, R.meta_vector(st.mel_len, s["texts"].device)

    def _capture(self, fn):
        """Warm fn up on a side stream (allocates per-stream workspaces outside the capture), then
        capture it there; returns (graph, outputs)."""
        dev = torch.device("cuda", torch.cuda.current_device())
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream(dev).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s, capture_error_mode="thread_local"):
            out = fn()
        self.captures += 1
        return graph, out

    def __call__(self, speakers, emotions, arousals, valences, texts, src_lens, max_src_len, p_targets=None,
                 e_targets=None, p_control=1.0, e_control=1.0, d_control=1.0):
        model = self.model
        dev = texts.device
        if dev.type != "cuda" or model.training:
            raise RuntimeError("SynthGraphs: eval-mode synthesis on a ROCm device")
        P = model.packed(dev)
        va = model.variance_adaptor
        B, Lx = texts.shape[0], int(max_src_len)
        if texts.shape[1] != Lx or B == 0:
            raise RuntimeError(f"SynthGraphs: texts {tuple(texts.shape)} vs max_src_len {Lx}")
        controls = (float(p_control), float(e_control), float(d_control))
        x = self._inputs(dev, speakers, emotions, arousals, valences, texts, src_lens, p_targets, e_targets)
        key1 = (model._precision, model._vp_precision, B, Lx, controls,
                tuple(k for k, v in x.items() if v is None))
        ops.bad_id_counter(dev)  # allocated outside any capture
        e1 = self._g1.get(key1)
        if e1 is not None and e1.P is not P:
            # the weights changed (a new pack): the graphs point at the old buffers. Drop this
            # stage-1 graph and every stage-2 graph that reads its outputs before recapturing.
            self._drop_stage1(key1)
            e1 = None
        if e1 is None:
            static = {k: (None if v is None else v.clone()) for k, v in x.items()}
            graph, (g, st, src_masks, meta) = self._capture(lambda: self._stage1_body(P, va, static, Lx, controls))
            meta_host = torch.empty(meta.shape, dtype=meta.dtype, pin_memory=True)
            e1 = self._g1[key1] = SimpleNamespace(graph=graph, static=static, g=g, st=st, src_masks=src_masks,
                                                  meta=meta, meta_host=meta_host, meta_np=meta_host.numpy(), P=P)
            while len(self._g1) > self.max_stage1:
                self._drop_stage1(next(iter(self._g1)))
        else:
            self._g1.move_to_end(key1)
        ks = [k for k, v in x.items() if v is not None]
        torch._foreach_copy_([e1.static[k] for k in ks], [x[k] for k in ks], non_blocking=True)  # one launch
        cur = torch.cuda.current_stream(dev)
        e1.graph.replay()
        # the one host read: the copy lands in pinned memory whose first entry (max mel_len >= 0)
        # the host set to -1; spinning on it returns as soon as the bytes land (a blocking
        # synchronize parks the thread and the wake-up cost ~30-60 us per call); the event
        # synchronize after it then returns at once and orders the rest of the copy (an event, not
        # the stream: the speculative decoder is queued behind it)
        e1.meta_np[0] = -1
        e1.meta_host.copy_(e1.meta, non_blocking=True)
        ev = getattr(e1, "ev", None)
        if ev is None:
            ev = e1.ev = torch.cuda.Event()
        ev.record(cur)
        st = e1.st
        packed = R.packed_stage2_ok(P, st, st.x)
        spec = None
        if packed and self.speculate:
            sk = self._spec_key(key1)
            if sk is not None:
                e2s = self._g2.get(key1 + ("dec", sk[0], sk[1]))
                if e2s is not None and e2s.e1 is e1 and e2s.graph_b is None:
                    e2s.graph.replay()  # under the host read
                    spec = (sk, e2s)
        _spin_until_landed(e1.meta_np)
        ev.synchronize()
        R.HOST_READS[0] += 1
        T_out, sum_len = R.check_meta(e1.meta_np, dev)
        pn_valid = R.postnet_valid_rows(B, T_out, sum_len)
        if packed:
            # the decoder graph per T bucket (T <= the stored PE table: no per-length recompute)
            T_b = -(-T_out // self.t_step) * self.t_step
            if T_b > P.dec_pe.shape[0]:
                T_b = T_out
            # the decoder's packed launches are sized from the bucketed row count (runtime.decode_packed)
            rows_b = ops.rows_bucket(sum_len, B * T_b)
            forms = R.decoder_forms(P, rows_b)
            if spec is not None:
                (T_s, rows_s, forms_s), e2s = spec
                hit = T_out <= T_s and sum_len <= rows_s and forms_s == forms
                self.spec_hits += hit
                self.spec_misses += not hit
            self._hist.setdefault(key1, deque(maxlen=self._history)).append((T_b, rows_b, forms))
            if spec is not None and hit:
                self._g2.move_to_end(key1 + ("dec", T_s, rows_s))
                e2 = e2s
            else:
                e2 = self._packed_entry(key1, e1, P, T_b, rows_b)
                e2.graph.replay()
                if e2.graph_b is not None:
                    e2.graph_b.replay()
            out = self._finish(e1, e2, cur, B, T_out, pn_valid, sum_len, src_lens, dev)
            if self.speculate:
                # the next call's speculation graph, captured now if the history moved it (so a serving
                # loop over a fixed set of batches stops capturing after one pass)
                sk = self._spec_key(key1)
                if not R.split_stage2_ok(P):
                    self._packed_entry(key1, e1, P, sk[0], sk[1])
            return out
        key2 = key1 + (T_out, pn_valid, ops.rows_bucket(sum_len, B * T_out))
        e2 = self._g2.get(key2)
        if e2 is not None and e2.e1 is not e1:  # captured on another (dropped) stage-1 entry's buffers
            del self._g2[key2]
            e2 = None
        if e2 is None:
            def body():
                mel, post, st2 = R._stage2(P, e1.g, st, T_out, T_out, controls[0], pn_valid, sum_len)
                return mel, post, R._mask(st2.mel_len, T_out)
            graph, outs = self._capture(body)
            e2 = self._g2[key2] = SimpleNamespace(graph=graph, graph_b=None, outs=outs, e1=e1)
            while len(self._g2) > self.max_stage2:
                self._g2.popitem(last=False)
        else:
            self._g2.move_to_end(key2)
        e2.graph.replay()
        outs = _fresh([st.p_pred, st.e_pred, st.log_d, st.d_rounded, e1.src_masks, st.mel_len] + list(e2.outs))
        p_pred, e_pred, log_d, d_rounded, src_masks, mel_len, mel, post, mel_masks = outs
        return (mel, post, p_pred, e_pred, log_d, d_rounded, src_masks, mel_masks, src_lens.to(dev), mel_len)

    def _packed_entry(self, key1, e1, P, T_b, rows_b):
        """The decoder graph(s) of (T bucket, row bucket) on stage-1 entry e1, captured if missing."""
        key2 = key1 + ("dec", T_b, rows_b)
        e2 = self._g2.get(key2)
        if e2 is not None and e2.e1 is not e1:  # captured on another (dropped) stage-1 entry's buffers
            del self._g2[key2]
            e2 = None
        if e2 is not None:
            self._g2.move_to_end(key2)
            return e2
        st = e1.st
        graph_b = None
        if R.split_stage2_ok(P):
            # two graphs: the LR launch + the first decoder block, then the other blocks. The first
            # replays (its outputs are the second's inputs: the second's warm-up run reads them),
            # then the second is captured
            graph, (x1, lay1, qkv1) = self._capture(lambda: R.decode_packed_head(P, st, st.x, st.mel_len, T_b, rows_b))
            graph.replay()
            graph_b, x_dec = self._capture(lambda: R.decode_packed_rest(P, x1, lay1, qkv1))
            outs = (x_dec, lay1)
        else:
            graph, outs = self._capture(lambda: R.decode_packed(P, st, st.x, st.mel_len, T_b, rows_b))
        e2 = self._g2[key2] = SimpleNamespace(graph=graph, graph_b=graph_b, outs=outs, e1=e1)
        while len(self._g2) > self.max_stage2:
            self._g2.popitem(last=False)
        return e2

    @staticmethod
    def _finish(e1, e2, cur, B, T_out, pn_valid, sum_len, src_lens, dev):
        """Behind the decoder graph on the caller's stream: fresh copies of stage 1's outputs (its
        buffers are overwritten by the next call's replay; one launch) and the T_out-shaped tail,
        eager (fresh outputs; the host enqueues it while the GPU runs the decoder). The decoder rows
        are read before the next call's replay overwrites them (same stream)."""
        st = e1.st
        p_pred, e_pred, log_d, d_rounded, src_masks, mel_len = _fresh(
            [st.p_pred, st.e_pred, st.log_d, st.d_rounded, e1.src_masks, st.mel_len])
        x_dec, _ = e2.outs
        lens = st.mel_len  # stage 1's buffer: read here, before the next call's replay
        lay = ops.SeqLayout(lens, T_out)
        mel, post = R.mel_postnet(e1.P, x_dec, lay, lens, pn_valid, sum_len)
        mel_masks = R._mask(lens, T_out)
        return (mel, post, p_pred, e_pred, log_d, d_rounded, src_masks, mel_masks, src_lens.to(dev), mel_len)
