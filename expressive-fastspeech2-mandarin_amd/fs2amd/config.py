"""Hyper-parameters of the mel-synthesis path and the preprocessed-data side files.

The schema is the reference's three YAMLs (``config/ESD-Chinese-Singing-MFA/{model,
preprocess,train}.yaml``); only the keys the forward path reads are used:

* ``model.yaml`` ``transformer.*``, ``variance_predictor.*``, ``variance_embedding.*``,
  ``multi_speaker``, ``multi_emotion``, ``max_seq_len`` (ref ``model/fastspeech2.py:16-71``,
  ``transformer/Models.py:36-52,106-119``, ``model/modules.py:20-55,200-213``)
* ``preprocess.yaml`` ``preprocessing.mel.n_mel_channels``, ``preprocessing.{pitch,energy}.feature``
  and ``path.preprocessed_path`` (``stats.json``, ``speakers.json``, ``emotions.json``).

The dictionaries below restate the ESD-Chinese-Singing-MFA values so the bench and the
GPU tests need no YAML files and no access to the reference tree.
"""
import copy
import json
import os

# ref config/ESD-Chinese-Singing-MFA/model.yaml:1-31
ESD_MODEL_CONFIG = {
    "transformer": {
        "encoder_layer": 4,
        "encoder_head": 2,
        "encoder_hidden": 256,
        "decoder_layer": 6,
        "decoder_head": 2,
        "decoder_hidden": 256,
        "conv_filter_size": 1024,
        "conv_kernel_size": [9, 1],
        "encoder_dropout": 0.2,
        "decoder_dropout": 0.2,
    },
    "variance_predictor": {"filter_size": 256, "kernel_size": 3, "dropout": 0.5},
    "variance_embedding": {
        "pitch_quantization": "linear",
        "energy_quantization": "linear",
        "n_bins": 256,
    },
    "multi_speaker": True,
    "multi_emotion": True,
    "max_seq_len": 2000,
    "vocoder": {"model": "HiFi-GAN", "speaker": "universal"},
}

# ref config/ESD-Chinese-Singing-MFA/preprocess.yaml (the keys the model reads)
ESD_PREPROCESS_CONFIG = {
    "dataset": "ESD-Chinese-Singing-MFA",
    "path": {"preprocessed_path": None},
    "preprocessing": {
        "val_size": 512,
        "text": {"text_cleaners": ["basic_cleaners"], "language": "zh"},
        "audio": {"sampling_rate": 22050, "max_wav_value": 32768.0},
        "stft": {"filter_length": 1024, "hop_length": 256, "win_length": 1024},
        "mel": {"n_mel_channels": 80, "mel_fmin": 0, "mel_fmax": 8000},
        "pitch": {"feature": "phoneme_level", "normalization": True},
        "energy": {"feature": "phoneme_level", "normalization": True},
    },
}

# ref config/ESD-Chinese-Singing-MFA/train.yaml:5-20
ESD_TRAIN_CONFIG = {
    "path": {"ckpt_path": "./output/ckpt", "log_path": "./output/log", "result_path": "./output/result"},
    "optimizer": {
        "batch_size": 4,
        "betas": [0.9, 0.98],
        "eps": 0.000000001,
        "weight_decay": 0.0,
        "grad_clip_thresh": 1.0,
        "grad_acc_step": 1,
        "warm_up_step": 4000,
        "anneal_steps": [300000, 400000, 500000],
        "anneal_rate": 0.3,
    },
    "step": {"total_step": 900000, "log_step": 100, "synth_step": 1000, "val_step": 1000, "save_step": 100000},
}

# Side files the survey fixes for synthetic runs: stats pitch=[-2,8,200,50],
# energy=[-1.5,9,40,20]; 10 speakers; 5 emotions / 4 arousal / 5 valence classes.
SYNTH_STATS = {"pitch": [-2.0, 8.0, 200.0, 50.0], "energy": [-1.5, 9.0, 40.0, 20.0]}
SYNTH_SPEAKERS = {f"spk{i:04d}": i for i in range(10)}
SYNTH_EMOTIONS = {
    "emotion_dict": {e: i for i, e in enumerate(["Angry", "Happy", "Neutral", "Sad", "Surprise"])},
    "arousal_dict": {a: i for i, a in enumerate(["0.3", "0.5", "0.8", "0.9"])},
    "valence_dict": {v: i for i, v in enumerate(["0.1", "0.2", "0.5", "0.6", "0.8"])},
}

# Vocabulary size: len(text.symbols_ipa.symbols) + 1 = 138 + 1 (ref transformer/Models.py:40,
# text/symbols_ipa.py:12-18). Pinyin phoneme ids used by the synthetic batches: 64..107.
N_SRC_VOCAB = 139


def write_side_files(directory, stats=None, speakers=None, emotions=None):
    """Write ``stats.json``, ``speakers.json`` and ``emotions.json`` into ``directory``."""
    os.makedirs(directory, exist_ok=True)
    with open(os.path.join(directory, "stats.json"), "w") as f:
        json.dump(stats or SYNTH_STATS, f)
    with open(os.path.join(directory, "speakers.json"), "w") as f:
        json.dump(speakers or SYNTH_SPEAKERS, f)
    with open(os.path.join(directory, "emotions.json"), "w") as f:
        json.dump(emotions or SYNTH_EMOTIONS, f)
    return directory


def synthetic_configs(preprocessed_path):
    """(preprocess_config, model_config, train_config) for a synthetic ESD run."""
    pc = copy.deepcopy(ESD_PREPROCESS_CONFIG)
    pc["path"]["preprocessed_path"] = preprocessed_path
    return pc, copy.deepcopy(ESD_MODEL_CONFIG), copy.deepcopy(ESD_TRAIN_CONFIG)
