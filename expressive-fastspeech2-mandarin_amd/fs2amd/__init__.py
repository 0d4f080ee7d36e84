"""fs2amd — MI355X-native FastSpeech2 mel-synthesis forward (HIP/CDNA4 kernels behind a C ABI).

    from fs2amd import FastSpeech2          # drop-in for the reference model/fastspeech2.py
"""
from .loss import FastSpeech2Loss
from .model import FastSpeech2, LengthRegulator
from .optimizer import ScheduledOptim

__all__ = ["FastSpeech2", "FastSpeech2Loss", "ScheduledOptim", "LengthRegulator"]
