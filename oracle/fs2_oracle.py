"""ORACLE — test infrastructure only. Never imported by the product path.

CPU restatement (PyTorch fp32, the same ATen ops in the same order) of the reference's
FastSpeech2 mel-synthesis forward, eval mode. It is the checker for the HIP path: only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.

Pinned: ``tests/test_oracle_golden.py`` checks it bit-for-bit against golden vectors that
``tests/golden/gen_golden.py`` captured by importing and running the reference itself
(Napoliee/Expressive-FastSpeech2-Mandarin @ /root/reference) in the build container.

Every function cites the reference file:line it restates. Parameters come in as a plain
``{state_dict key: CPU float tensor}`` mapping (the reference's 240 keys).
"""
import numpy as np
import torch
import torch.nn.functional as F


# ---------------------------------------------------------------- helpers
def sinusoid_table(n_position, d_hid):
    """ref transformer/Models.py:10-30 (numpy fp64 -> torch.FloatTensor)."""
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    hid = np.arange(d_hid)
    angle = pos / np.power(10000, 2 * (hid // 2) / d_hid)
    table = np.array(angle)
    table[:, 0::2] = np.sin(table[:, 0::2])
    table[:, 1::2] = np.cos(table[:, 1::2])
    return torch.FloatTensor(table)


def mask_from_lengths(lengths, max_len=None):
    """ref utils/tools.py:152-160 (True = padding)."""
    batch_size = lengths.shape[0]
    if max_len is None:
        max_len = torch.max(lengths).item()
    ids = torch.arange(0, max_len).unsqueeze(0).expand(batch_size, -1)
    return ids >= lengths.unsqueeze(1).expand(-1, max_len)


def pad_frames(seqs, max_len=None):
    """ref utils/tools.py:360-378 (2-D branch; negative pad crops)."""
    if max_len:
        target = max_len
    else:
        target = max(s.size(0) for s in seqs)
    return torch.stack([F.pad(s, (0, 0, 0, target - s.size(0)), "constant", 0.0) for s in seqs])


# ---------------------------------------------------------------- transformer blocks
def multi_head_attention(sd, pre, x, slf_mask, n_head):
    """ref transformer/SubLayers.py:29-57 + Modules.py:14-25 (dropout = identity in eval)."""
    sz_b, len_q, d_model = x.size()
    d_k = d_model // n_head
    residual = x
    q = F.linear(x, sd[pre + "w_qs.weight"], sd[pre + "w_qs.bias"]).view(sz_b, len_q, n_head, d_k)
    k = F.linear(x, sd[pre + "w_ks.weight"], sd[pre + "w_ks.bias"]).view(sz_b, len_q, n_head, d_k)
    v = F.linear(x, sd[pre + "w_vs.weight"], sd[pre + "w_vs.bias"]).view(sz_b, len_q, n_head, d_k)
    q = q.permute(2, 0, 1, 3).contiguous().view(-1, len_q, d_k)
    k = k.permute(2, 0, 1, 3).contiguous().view(-1, len_q, d_k)
    v = v.permute(2, 0, 1, 3).contiguous().view(-1, len_q, d_k)
    mask = slf_mask.repeat(n_head, 1, 1)
    attn = torch.bmm(q, k.transpose(1, 2))
    attn = attn / np.power(d_k, 0.5)
    attn = attn.masked_fill(mask, -np.inf)
    attn = torch.softmax(attn, dim=2)
    out = torch.bmm(attn, v)
    out = out.view(n_head, sz_b, len_q, d_k).permute(1, 2, 0, 3).contiguous().view(sz_b, len_q, -1)
    out = F.linear(out, sd[pre + "fc.weight"], sd[pre + "fc.bias"])
    return F.layer_norm(out + residual, (d_model,), sd[pre + "layer_norm.weight"], sd[pre + "layer_norm.bias"])


def positionwise_ffn(sd, pre, x, kernel_size):
    """ref transformer/SubLayers.py:85-93."""
    residual = x
    out = x.transpose(1, 2)
    out = F.conv1d(out, sd[pre + "w_1.weight"], sd[pre + "w_1.bias"], padding=(kernel_size[0] - 1) // 2)
    out = F.conv1d(F.relu(out), sd[pre + "w_2.weight"], sd[pre + "w_2.bias"], padding=(kernel_size[1] - 1) // 2)
    out = out.transpose(1, 2)
    return F.layer_norm(out + residual, (x.size(-1),), sd[pre + "layer_norm.weight"], sd[pre + "layer_norm.bias"])


def fft_block(sd, pre, x, mask, slf_mask, n_head, kernel_size):
    """ref transformer/Layers.py:21-30."""
    out = multi_head_attention(sd, pre + "slf_attn.", x, slf_mask, n_head)
    out = out.masked_fill(mask.unsqueeze(-1), 0)
    out = positionwise_ffn(sd, pre + "pos_ffn.", out, kernel_size)
    return out.masked_fill(mask.unsqueeze(-1), 0)


def encoder(sd, cfg, src_seq, mask, training=False):
    """ref transformer/Models.py:73-100 (dropout identity; training only changes the PE rule :82)."""
    tr = cfg["transformer"]
    batch_size, max_len = src_seq.shape
    slf_mask = mask.unsqueeze(1).expand(-1, max_len, -1)
    emb = F.embedding(src_seq, sd["encoder.src_word_emb.weight"], padding_idx=0)
    if not training and max_len > cfg["max_seq_len"]:
        pe = sinusoid_table(max_len, tr["encoder_hidden"])[:max_len, :].unsqueeze(0).expand(batch_size, -1, -1)
    else:
        pe = sd["encoder.position_enc"][:, :max_len, :].expand(batch_size, -1, -1)
    out = emb + pe
    for i in range(tr["encoder_layer"]):
        out = fft_block(sd, f"encoder.layer_stack.{i}.", out, mask, slf_mask, tr["encoder_head"], tr["conv_kernel_size"])
    return out


def decoder(sd, cfg, enc_seq, mask, training=False):
    """ref transformer/Models.py:139-171 (dropout identity; training crops to max_seq_len, :145-162)."""
    tr = cfg["transformer"]
    batch_size, max_len = enc_seq.shape[0], enc_seq.shape[1]
    if not training and max_len > cfg["max_seq_len"]:
        slf_mask = mask.unsqueeze(1).expand(-1, max_len, -1)
        out = enc_seq + sinusoid_table(max_len, tr["decoder_hidden"])[:max_len, :].unsqueeze(0).expand(batch_size, -1, -1)
    else:
        max_len = min(max_len, cfg["max_seq_len"])
        slf_mask = mask.unsqueeze(1).expand(-1, max_len, -1)
        out = enc_seq[:, :max_len, :] + sd["decoder.position_enc"][:, :max_len, :].expand(batch_size, -1, -1)
        mask = mask[:, :max_len]
        slf_mask = slf_mask[:, :, :max_len]
    for i in range(tr["decoder_layer"]):
        out = fft_block(sd, f"decoder.layer_stack.{i}.", out, mask, slf_mask, tr["decoder_head"], tr["conv_kernel_size"])
    return out, mask


def postnet(sd, x, training=False):
    """ref transformer/Layers.py:129-137 (+ ConvNorm :33-64; dropout identity). training: BatchNorm1d
    uses batch statistics over (B, T) and updates the running buffers in ``sd`` in place."""
    x = x.contiguous().transpose(1, 2)
    n = 5
    for i in range(n):
        pre = f"postnet.convolutions.{i}."
        y = F.conv1d(x, sd[pre + "0.conv.weight"], sd[pre + "0.conv.bias"], padding=2)
        y = F.batch_norm(y, sd[pre + "1.running_mean"], sd[pre + "1.running_var"], sd[pre + "1.weight"],
                         sd[pre + "1.bias"], training, 0.1, 1e-5)
        x = torch.tanh(y) if i < n - 1 else y
    return x.contiguous().transpose(1, 2)


# ---------------------------------------------------------------- variance adaptor
def variance_predictor(sd, pre, x, mask):
    """ref model/modules.py:209-250 (+ Conv :253-296); conv1d_2 padding hard-coded to 1 (:230)."""
    d = x.size(-1)
    out = x.contiguous().transpose(1, 2)
    out = F.conv1d(out, sd[pre + "conv_layer.conv1d_1.conv.weight"], sd[pre + "conv_layer.conv1d_1.conv.bias"], padding=1)
    out = out.contiguous().transpose(1, 2)
    out = F.layer_norm(F.relu(out), (d,), sd[pre + "conv_layer.layer_norm_1.weight"], sd[pre + "conv_layer.layer_norm_1.bias"])
    out = out.contiguous().transpose(1, 2)
    out = F.conv1d(out, sd[pre + "conv_layer.conv1d_2.conv.weight"], sd[pre + "conv_layer.conv1d_2.conv.bias"], padding=1)
    out = out.contiguous().transpose(1, 2)
    out = F.layer_norm(F.relu(out), (d,), sd[pre + "conv_layer.layer_norm_2.weight"], sd[pre + "conv_layer.layer_norm_2.bias"])
    out = F.linear(out, sd[pre + "linear_layer.weight"], sd[pre + "linear_layer.bias"]).squeeze(-1)
    if mask is not None:
        out = out.masked_fill(mask, 0.0)
    return out


def variance_embedding(sd, kind, x, target, mask, control):
    """ref model/modules.py:80-100 (get_pitch_embedding / get_energy_embedding)."""
    prediction = variance_predictor(sd, f"variance_adaptor.{kind}_predictor.", x, mask)
    bins = sd[f"variance_adaptor.{kind}_bins"]
    table = sd[f"variance_adaptor.{kind}_embedding.weight"]
    if target is not None:
        embedding = F.embedding(torch.bucketize(target, bins), table)
    else:
        prediction = prediction * control
        embedding = F.embedding(torch.bucketize(prediction, bins), table)
    return prediction, embedding


def length_regulate(x, duration, max_len):
    """ref model/modules.py:167-194 (LR / expand / forward). Returns (out, mel_len int64)."""
    output, mel_len = [], []
    for batch, expand_target in zip(x, duration):
        pieces = []
        for i, vec in enumerate(batch):
            expand_size = expand_target[i].item()
            pieces.append(vec.expand(max(int(expand_size), 0), -1))
        expanded = torch.cat(pieces, 0)
        output.append(expanded)
        mel_len.append(expanded.shape[0])
    out = pad_frames(output, max_len) if max_len is not None else pad_frames(output)
    return out, torch.LongTensor(mel_len)


def length_regulate_index_map(duration, max_len):
    """Source-phoneme index per output frame (-1 = padding), derived through the very same
    expand/cat/pad sequence as :func:`length_regulate` on an index-valued input."""
    B, L = duration.shape
    idx = (torch.arange(L, dtype=torch.float64) + 1).view(1, L, 1).expand(B, L, 1).contiguous()
    out, mel_len = length_regulate(idx, duration, max_len)
    return (out[..., 0].round().to(torch.int64) - 1).to(torch.int32), mel_len


def variance_adaptor(sd, cfg, pcfg, x, src_mask, mel_mask, max_len, p_t, e_t, d_t, p_c, e_c, d_c):
    """ref model/modules.py:102-158 (phoneme-level pitch/energy; energy uses p_control, :124-125)."""
    log_d = variance_predictor(sd, "variance_adaptor.duration_predictor.", x, src_mask)
    p_level = pcfg["preprocessing"]["pitch"]["feature"]
    e_level = pcfg["preprocessing"]["energy"]["feature"]
    p_pred = e_pred = None
    if p_level == "phoneme_level":
        p_pred, p_emb = variance_embedding(sd, "pitch", x, p_t, src_mask, p_c)
        x = x + p_emb
    if e_level == "phoneme_level":
        e_pred, e_emb = variance_embedding(sd, "energy", x, e_t, src_mask, p_c)
        x = x + e_emb
    if d_t is not None:
        x, mel_len = length_regulate(x, d_t, max_len)
        d_rounded = d_t
    else:
        d_rounded = torch.clamp(torch.round(torch.exp(log_d) - 1) * d_c, min=0)
        x, mel_len = length_regulate(x, d_rounded, max_len)
        mel_mask = mask_from_lengths(mel_len)
    if p_level == "frame_level":
        p_pred, p_emb = variance_embedding(sd, "pitch", x, p_t, mel_mask, p_c)
        x = x + p_emb
    if e_level == "frame_level":
        e_pred, e_emb = variance_embedding(sd, "energy", x, e_t, mel_mask, p_c)
        x = x + e_emb
    return x, p_pred, e_pred, log_d, d_rounded, mel_len, mel_mask


# ---------------------------------------------------------------- top level
def forward(sd, model_config, preprocess_config, speakers, emotions, arousals, valences, texts, src_lens,
            max_src_len, mels=None, mel_lens=None, max_mel_len=None, p_targets=None, e_targets=None,
            d_targets=None, p_control=1.0, e_control=1.0, d_control=1.0, training=False):
    """ref model/fastspeech2.py:73-148. Returns the reference's 10-tuple. ``training``: train-mode
    semantics with every dropout disabled (BN batch statistics, decoder crop), differentiable."""
    cfg = model_config
    src_masks = mask_from_lengths(src_lens, max_src_len)
    mel_masks = mask_from_lengths(mel_lens, max_mel_len) if mel_lens is not None else None
    output = encoder(sd, cfg, texts, src_masks, training)
    if cfg["multi_speaker"]:
        output = output + F.embedding(speakers, sd["speaker_emb.weight"]).unsqueeze(1).expand(-1, max_src_len, -1)
    if cfg["multi_emotion"]:
        emb = torch.cat((F.embedding(emotions, sd["emotion_emb.weight"]), F.embedding(arousals, sd["arousal_emb.weight"]),
                         F.embedding(valences, sd["valence_emb.weight"])), dim=-1)
        cond = F.relu(F.linear(emb, sd["emotion_linear.0.weight"], sd["emotion_linear.0.bias"]))
        output = output + cond.unsqueeze(1).expand(-1, max_src_len, -1)
    (output, p_pred, e_pred, log_d, d_rounded, mel_lens, mel_masks) = variance_adaptor(
        sd, cfg, preprocess_config, output, src_masks, mel_masks, max_mel_len, p_targets, e_targets, d_targets,
        p_control, e_control, d_control)
    output, mel_masks = decoder(sd, cfg, output, mel_masks, training)
    output = F.linear(output, sd["mel_linear.weight"], sd["mel_linear.bias"])
    postnet_output = postnet(sd, output, training) + output
    return (output, postnet_output, p_pred, e_pred, log_d, d_rounded, src_masks, mel_masks, src_lens, mel_lens)


def loss(preprocess_config, mels, pitches, energies, durations, predictions):
    """ref model/loss.py:19-92: (total, mel L1, postnet L1, pitch MSE, energy MSE, log-duration MSE)
    over un-padded positions; mel targets cropped to the prediction's frames (:41-42)."""
    mel_pred, post_pred, p_pred, e_pred, log_d, _, src_masks, mel_masks, _, _ = predictions
    src_valid, mel_valid = ~src_masks, ~mel_masks
    log_d_t = torch.log(durations.float() + 1)
    mels = mels[:, : mel_valid.shape[1], :]
    sel = lambda lvl: src_valid if lvl == "phoneme_level" else mel_valid
    pp = preprocess_config["preprocessing"]
    p_m, e_m = sel(pp["pitch"]["feature"]), sel(pp["energy"]["feature"])
    mv = mel_valid.unsqueeze(-1)
    mel_l = F.l1_loss(mel_pred.masked_select(mv), mels.masked_select(mv))
    post_l = F.l1_loss(post_pred.masked_select(mv), mels.masked_select(mv))
    p_l = F.mse_loss(p_pred.masked_select(p_m), pitches.masked_select(p_m))
    e_l = F.mse_loss(e_pred.masked_select(e_m), energies.masked_select(e_m))
    d_l = F.mse_loss(log_d.masked_select(src_valid), log_d_t.masked_select(src_valid))
    return mel_l + post_l + d_l + p_l + e_l, mel_l, post_l, p_l, e_l, d_l


def build_state_dict(model_config, preprocess_config, stats, generated):
    """Assemble the full 240-key mapping: generated tensors + the constructor-computed ones
    (PE tables ref transformer/Models.py:59-62,125-128; bins ref model/modules.py:41-71)."""
    sd = {k: torch.as_tensor(v) for k, v in generated.items()}
    n_pos = model_config["max_seq_len"] + 1
    tr = model_config["transformer"]
    sd["encoder.position_enc"] = sinusoid_table(n_pos, tr["encoder_hidden"]).unsqueeze(0)
    sd["decoder.position_enc"] = sinusoid_table(n_pos, tr["decoder_hidden"]).unsqueeze(0)
    n_bins = model_config["variance_embedding"]["n_bins"]
    for kind in ("pitch", "energy"):
        lo, hi = stats[kind][:2]
        if model_config["variance_embedding"][f"{kind}_quantization"] == "log":
            bins = torch.exp(torch.linspace(np.log(lo), np.log(hi), n_bins - 1))
        else:
            bins = torch.linspace(lo, hi, n_bins - 1)
        sd[f"variance_adaptor.{kind}_bins"] = bins
    for i in range(5):
        sd[f"postnet.convolutions.{i}.1.num_batches_tracked"] = torch.tensor(0)
    return sd
