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
        self.mse_loss = nn.MSELoss()
        self.mae_loss = nn.L1Loss()

    def forward(self, inputs, predictions):
        mel_targets, _, _, pitch_targets, energy_targets, duration_targets = inputs[9:]
        (mel_pred, postnet_pred, pitch_pred, energy_pred, log_d_pred, _, src_masks, mel_masks, _, _) = predictions
        src_valid = ~src_masks
        mel_valid = ~mel_masks
        log_d_targets = torch.log(duration_targets.float() + 1).detach()
        mel_targets = mel_targets[:, : mel_valid.shape[1], :].detach()
        pitch_targets, energy_targets = pitch_targets.detach(), energy_targets.detach()

        def sel(level, pred, tgt):
            m = src_valid if level == "phoneme_level" else mel_valid
            return pred.masked_select(m), tgt.masked_select(m)

        pitch_pred, pitch_targets = sel(self.pitch_feature_level, pitch_pred, pitch_targets)
        energy_pred, energy_targets = sel(self.energy_feature_level, energy_pred, energy_targets)
        log_d_pred = log_d_pred.masked_select(src_valid)
        log_d_targets = log_d_targets.masked_select(src_valid)
        mv = mel_valid.unsqueeze(-1)
        mel_pred = mel_pred.masked_select(mv)
        postnet_pred = postnet_pred.masked_select(mv)
        mel_targets = mel_targets.masked_select(mv)

        mel_loss = self.mae_loss(mel_pred, mel_targets)
        postnet_mel_loss = self.mae_loss(postnet_pred, mel_targets)
        pitch_loss = self.mse_loss(pitch_pred, pitch_targets)
        energy_loss = self.mse_loss(energy_pred, energy_targets)
        duration_loss = self.mse_loss(log_d_pred, log_d_targets)
        total = mel_loss + postnet_mel_loss + duration_loss + pitch_loss + energy_loss
        return total, mel_loss, postnet_mel_loss, pitch_loss, energy_loss, duration_loss
