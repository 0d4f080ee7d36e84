"""Drop-in for the reference's ``model`` package (model/__init__.py:1-3): put
``expressive-fastspeech2-mandarin_amd/`` on sys.path ahead of the reference tree and
``from model import FastSpeech2, FastSpeech2Loss, ScheduledOptim`` resolves here. Importing it also
registers the hot-path ops as ``torch.ops.fs2.*`` (fs2amd.library: torch.library custom ops with
fake implementations, so torch.compile / torch.export trace through them)."""
import fs2amd.library  # noqa: F401  (registers torch.ops.fs2.*)
from fs2amd.loss import FastSpeech2Loss
from fs2amd.model import FastSpeech2, LengthRegulator
from fs2amd.optimizer import ScheduledOptim

__all__ = ["FastSpeech2", "FastSpeech2Loss", "ScheduledOptim", "LengthRegulator"]
