"""Drop-in for the reference's ``model`` package (model/__init__.py:1-3): put
``expressive-fastspeech2-mandarin_amd/`` on sys.path ahead of the reference tree and
``from model import FastSpeech2, FastSpeech2Loss, ScheduledOptim`` resolves here."""
from fs2amd.loss import FastSpeech2Loss
from fs2amd.model import FastSpeech2, LengthRegulator
from fs2amd.optimizer import ScheduledOptim

__all__ = ["FastSpeech2", "FastSpeech2Loss", "ScheduledOptim", "LengthRegulator"]
