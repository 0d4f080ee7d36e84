"""FastSpeech2Loss with the reference's semantics (model/loss.py:5-92).

(total, mel L1, postnet L1, pitch MSE, energy MSE, log-duration MSE) over the un-padded
positions; the mel target is cropped to the prediction's frame count first (:41-42).
"""
import torch
import torch.nn as nn


class FastSpeech2Loss(nn.Module):
    def __init__(self, preprocess_config, model_config):
        super().__init__()
        self.pitch_feature_level = preprocess_config["preprocessing"]["pitch"]["feature"]
        self.energy_feature_level = preprocess_config["preprocessing"]["energy"]["feature"]

    def forward(self, inputs, predictions):
        mel_targets, _, _, pitch_targets, energy_targets, duration_targets = inputs[9:]
        (mel_pred, postnet_pred, pitch_pred, energy_pred, log_d_pred, _, src_masks, mel_masks, _, _) = predictions
        src_valid = ~src_masks
        mel_valid = ~mel_masks
        log_d_targets = torch.log(duration_targets.float() + 1).detach()
        mel_targets = mel_targets[:, : mel_valid.shape[1], :].detach()
        pitch_targets, energy_targets = pitch_targets.detach(), energy_targets.detach()

        # masked means as sum(err * mask) / count: the same quantity as masked_select(...).mean()
        # (NaN for an empty selection, like the reference) without a data-dependent shape, so the
        # step has no host sync here
        def mmean(err, m):
            mf = m.to(err.dtype).expand_as(err)
            return (err * mf).sum() / mf.sum()

        sel = lambda level: src_valid if level == "phoneme_level" else mel_valid
        mv = mel_valid.unsqueeze(-1)
        mel_loss = mmean((mel_pred - mel_targets).abs(), mv)
        postnet_mel_loss = mmean((postnet_pred - mel_targets).abs(), mv)
        pitch_loss = mmean((pitch_pred - pitch_targets) ** 2, sel(self.pitch_feature_level))
        energy_loss = mmean((energy_pred - energy_targets) ** 2, sel(self.energy_feature_level))
        duration_loss = mmean((log_d_pred - log_d_targets) ** 2, src_valid)
        total = mel_loss + postnet_mel_loss + duration_loss + pitch_loss + energy_loss
        return total, mel_loss, postnet_mel_loss, pitch_loss, energy_loss, duration_loss
